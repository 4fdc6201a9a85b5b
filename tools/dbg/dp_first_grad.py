"""Debug: first-step weight gradients, eager vs graph TrainStep (fp32, no process group)."""
import sys
import torch
from dcnn_amd.models import zoo
from dcnn_amd.nn import Adam, LossFactory
from dcnn_amd.runtime.step import TrainStep


def run(use_graph):
    m = zoo.create_model("resnet18_tiny_imagenet")
    m.set_seed(5)
    m.set_device("GPU:0")
    m.set_compute_dtype(torch.float32)
    m.initialize()
    m.set_first_layer_input_grad(False)
    opt = Adam(1e-3)
    opt.attach(m)
    st = TrainStep(m, LossFactory.create("softmax_crossentropy"), opt, use_graph=use_graph)
    g = torch.Generator().manual_seed(11)
    x = torch.randn(32, 3, 64, 64, generator=g).cuda()
    y = torch.randint(0, 200, (32,), generator=g).cuda()
    l0 = float(st(x, y))
    return l0, m.arena.grad.cpu(), m.arena.data.cpu()


le, ge, pe = run(False)
le2, ge2, pe2 = run(False)
lg, gg, pg = run(True)
print("loss eager", le, "eager2", le2, "graph", lg)
print("grad eager vs eager2", (ge - ge2).norm().item(), "eager vs graph", (ge - gg).norm().item(), "norm", ge.norm().item())
print("param eager vs graph", (pe - pg).norm().item())
