import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from torchbooster_amd.ops._ext import native
from torchbooster_amd.ops import conv as nc
def rel(a, b): return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()
torch.manual_seed(0)
dev = "cuda"
N, C, H, K = 4, 256, 16, 64
x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
w = (torch.randn(K, C, 1, 1, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
dy = torch.randn(N, K, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
add = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
wt = native().conv_flip_weight(w)
d0 = native().conv2d_fwd(dy, wt, None, 1, 0, False, False)[0]
d1 = native().conv2d_fwd(dy, wt, None, 1, 0, False, False, add)[0]
ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w.float(), None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False])[0]
print("dgrad", rel(d0, ref), "dgrad+add", rel(d1, ref + add.float()))
# passthrough through autograd
xa = x.clone().requires_grad_()
y, st, xp = nc.conv2d_bn_stats(xa, w, 1, 0, True)
(y.float() * dy.float()).sum().backward(retain_graph=True)
print("grad no pass", rel(xa.grad, ref))
xa.grad = None
y, st, xp = nc.conv2d_bn_stats(xa, w, 1, 0, True)
((y.float() * dy.float()).sum() + (xp.float() * add.float()).sum()).backward()
print("grad with pass", rel(xa.grad, ref + add.float()))
print(nc.autotune_table())
