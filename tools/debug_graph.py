import torch, sys
sys.path.insert(0, '.')
from dcnn_amd.ops import hip
p = torch.randn(8, 10, device='cuda')
lab = torch.randint(0, 10, (8,), device='cuda')
l, g, c = hip.loss_fused(p, None, lab)
print('eager loss', l.item())
s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    hip.loss_fused(p, None, lab)
torch.cuda.current_stream().wait_stream(s)
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    L, G, Cc = hip.loss_fused(p, None, lab)
for i in range(3):
    gr.replay(); torch.cuda.synchronize(); print('replay', i, L.item(), Cc.item())
# memset via torch zero_ inside graph for comparison
z = torch.ones(4, device='cuda')
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    z.zero_(); z.add_(1)
for i in range(3):
    g2.replay(); torch.cuda.synchronize(); print('torch zero replay', z.tolist())
