import torch
torch.manual_seed(0)
print("allow_tf32", torch.backends.cuda.matmul.allow_tf32, getattr(torch.backends.cuda.matmul, "fp32_precision", None))
for (b, n, k, m) in [(16, 256, 8, 256), (16, 256, 256, 64), (16, 1024, 1024, 128), (2, 256, 2, 256)]:
    a = torch.randn(b, n, k, device="cuda"); c = torch.randn(b, k, m, device="cuda")
    r = torch.bmm(a, c); r64 = torch.bmm(a.double(), c.double())
    print(b, n, k, m, ((r.double() - r64).norm() / r64.norm()).item())
