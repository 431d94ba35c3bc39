import torch, ctypes, os
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprobe.so"))
A = torch.randn(16, 32, device="cuda").bfloat16(); B = torch.randn(16, 32, device="cuda").bfloat16()
C = torch.empty(16, 16, device="cuda")
s = torch.cuda.current_stream().cuda_stream
r = lib.probe_mfma(ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(C.data_ptr()), ctypes.c_void_p(s))
torch.cuda.synchronize()
ref = A.float() @ B.float().t()
print("ret", r, "maxerr", (C - ref).abs().max().item(), torch.cuda.get_device_name(0))
