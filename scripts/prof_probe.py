import torch
x = torch.randn(1 << 20, device="cuda")
for _ in range(10):
    x = x * 1.0001 + 1
torch.cuda.synchronize()
print("probe ok", float(x.sum()))
