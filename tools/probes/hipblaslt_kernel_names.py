import torch
M,N,K=49020,4096,1024
a=torch.randn(M,K,device="cuda").bfloat16(); w=torch.randn(N,K,device="cuda").bfloat16()
for _ in range(5): torch.nn.functional.linear(a,w)
torch.cuda.synchronize()
a2=torch.randn(M,4096,device="cuda").bfloat16(); w2=torch.randn(1024,4096,device="cuda").bfloat16()
for _ in range(5): torch.nn.functional.linear(a2,w2)
torch.cuda.synchronize()
