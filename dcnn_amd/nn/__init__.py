"""Neural-network layer stack: layers, Sequential, losses, optimizers, schedulers."""
from .activations import ActivationFactory, ActivationFunction  # noqa: F401
from .layers import *  # noqa: F401,F403
from .loss import (CrossEntropyLoss, HuberLoss, LogSoftmaxCrossEntropyLoss, Loss, LossFactory,  # noqa: F401
                   MAELoss, MSELoss, SoftmaxCrossEntropyLoss)
from .optimizers import SGD, Adam, AdamW, Optimizer, OptimizerConfig, OptimizerFactory  # noqa: F401
from .params import ParamArena, ParamSpec  # noqa: F401
from .schedulers import *  # noqa: F401,F403
from .sequential import Partition, Sequential, SequentialBuilder, load_tensor, save_tensor  # noqa: F401
from .train import (TrainingConfig, load_checkpoint, save_checkpoint, train_class_epoch,  # noqa: F401
                    train_classification_model, train_reg_epoch, train_regression_model, validate_class_model,
                    validate_reg_model)
