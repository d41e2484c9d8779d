"""Diagnostic: the HIP conv stack (forward) against the fp32 torch model on one flagship batch."""
import os
import sys

import torch
import torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from quantum_distributed_machine_learning_ris_channel_estimation_amd.ops.conv import ConvStackHIP
from quantum_distributed_machine_learning_ris_channel_estimation_amd.train.engine import HDCEModel
cuda = torch.device('cuda')
def rel(a, b):
    b = b.detach().reshape(a.shape); return float((a.float()-b.float()).norm()/b.float().norm().clamp_min(1e-12))
torch.manual_seed(0)
U, B = 3, 256
a = HDCEModel(128, cuda, 'bf16'); b = HDCEModel(128, cuda, 'fp32')
with torch.no_grad():
    b.space.flat.copy_(a.space.flat)
Yp = torch.randn(3, U, B, 2, 16, 8, device=cuda)
conv = ConvStackHIP(a, U, B)
x1 = a.pack_input(Yp).contiguous()
h3 = conv.forward(x1, True)
# reference with retained intermediates
h = b.pack_input(Yp)
hs, zs = [], []
for k in range(3):
    z = F.conv2d(h, b.conv_w[k], padding=1, groups=3); z.retain_grad(); zs.append(z)
    h = b._ghost_bn_relu(z, k, U, True); h.retain_grad(); hs.append(h)
ref = h.reshape(U*B*3, -1)
print('fwd h3 rel', rel(h3, ref))
for k in range(3): print('z', k, rel(conv.z[k].float(), zs[k].detach().reshape(conv.z[k].shape)))
dh = torch.randn_like(ref)
a.space.zero_grad(); b.space.zero_grad()
conv.backward(dh.to(torch.bfloat16)); ref.backward(dh); torch.cuda.synchronize()
print('dx h2', rel(conv.dx[1], hs[1].grad), 'dx h1', rel(conv.dx[0], hs[0].grad))
for k in range(3):
    print(k, 'W', rel(a.conv_w[k].grad, b.conv_w[k].grad), 'g', rel(a.bn_w[k].grad, b.bn_w[k].grad), 'b', rel(a.bn_b[k].grad, b.bn_b[k].grad))
    print('   |Wgrad| a', a.conv_w[k].grad.norm().item(), 'b', b.conv_w[k].grad.norm().item())
# isolate layer-1 wgrad: feed the reference dL/dh1 (fp32) as upstream into a fresh backward of layer 1 only
print('bn st1 c consts sample', conv.st[0][0, :4].tolist())
