import torch
M,N,K=32768,4096,768
x=torch.randn(M,K,device="cuda").bfloat16(); w=torch.randn(N,K,device="cuda").bfloat16(); dy=torch.randn(M,N,device="cuda").bfloat16()
for _ in range(3):
    y=x@w.t(); z=dy@w; t=dy.t()@x
torch.cuda.synchronize()
