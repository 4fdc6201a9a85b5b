"""Debug: device Adam scalars across graph replays vs eager (fp32 ResNet-18, no process group)."""
import torch
from dcnn_amd.models import zoo
from dcnn_amd.nn import Adam, LossFactory
from dcnn_amd.runtime.step import TrainStep


def run(use_graph, steps=4):
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
    out = []
    for i in range(steps):
        l = float(st(x, y))
        torch.cuda.synchronize()
        out.append((round(l, 6), opt.t, [round(v, 6) for v in opt._hyper.cpu().tolist()]))
    return out


for ug in (False, True):
    print("graph" if ug else "eager")
    for r in run(ug):
        print("  ", r)
