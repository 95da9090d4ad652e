import sys, os, math, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from picotron_amd import kernels as K
dev = "cuda"
B, S, H, D = 1, 128, 1, 64
q = torch.zeros(B, S, H, D); k = torch.zeros(B, S, H, D)
v = torch.zeros(B, S, H, D)
# q=k=0 -> uniform attention (full): out[q][d] = mean_k v[k][d]; use v[k][d] = d so out = d exactly
v[..., :] = torch.arange(D).float()
o, lse = K.attn_fwd(q.to(torch.bfloat16).to(dev), k.to(torch.bfloat16).to(dev), v.to(torch.bfloat16).to(dev), 1.0, False)
print("uniform full, v=d: out row0", o[0, 0, 0, :16].tolist())
print("lse[0,0,:4]", lse[0, 0, :4].tolist(), "expected", math.log(S))
v2 = torch.zeros(B, S, H, D); v2[:, :, :, :] = torch.arange(S).float().view(1, S, 1, 1) / S
o, lse = K.attn_fwd(q.to(torch.bfloat16).to(dev), k.to(torch.bfloat16).to(dev), v2.to(torch.bfloat16).to(dev), 1.0, False)
print("uniform full, v=k/S: out row0", o[0, 0, 0, :8].tolist(), "expected", (torch.arange(S).float()/S).to(torch.bfloat16).float().mean().item())
# single key: k0 big dot with q -> out ~ v[k0]
q3 = torch.zeros(B, S, H, D); q3[..., 0] = 1
k3 = torch.zeros(B, S, H, D); k3[0, 37, 0, 0] = 30
v3 = torch.zeros(B, S, H, D); v3[0, 37, 0, :] = torch.arange(D).float()
o, lse = K.attn_fwd(q3.to(torch.bfloat16).to(dev), k3.to(torch.bfloat16).to(dev), v3.to(torch.bfloat16).to(dev), 1.0, False)
print("peaked key 37: out row5", o[0, 5, 0, :16].tolist())
