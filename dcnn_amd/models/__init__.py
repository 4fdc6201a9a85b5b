"""Model zoo (reference `include/nn/example_models.hpp`)."""
from .zoo import *  # noqa: F401,F403
from .zoo import MODELS, INPUT_SHAPES, NUM_CLASSES, create_model  # noqa: F401
