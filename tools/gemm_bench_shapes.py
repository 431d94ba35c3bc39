"""The model's conv GEMM shapes at B=16, 224^2 (shared by gemm_bench.py and blas_ref_bench.py)."""
# name, H, Cseg, nsrc, ntaps(1|9|11), N
SHAPES = [("L1 3x3 fwd up_conv1", 224, 64, 2, 9, 64), ("L1 3x3 dgrad up_conv1", 224, 64, 1, 11, 128),
          ("L1 1x1 gate", 224, 64, 2, 1, 64), ("L1 1x1 fusion", 224, 64, 3, 1, 64),
          ("L1 1x1 entry+res", 224, 64, 2, 1, 128), ("L1 3x3 down1 (Cin 8)", 224, 8, 1, 9, 64),
          ("L2 3x3 fwd up_conv2", 112, 128, 2, 9, 128), ("L2 3x3 dgrad", 112, 128, 1, 11, 256),
          ("L3 3x3 fwd up_conv3", 56, 256, 2, 9, 256), ("L4 3x3 fwd up_conv4", 28, 512, 2, 9, 512),
          ("BN 3x3 fwd bottleneck", 14, 512, 1, 9, 1024), ("L4 3x3 dgrad up_conv4", 28, 512, 1, 11, 1024),
          ("BN 3x3 dgrad bottleneck", 14, 1024, 1, 11, 512), ("L4 3x3 dgrad down4", 28, 512, 1, 11, 256),
          ("L2 3x3 dgrad N64", 112, 128, 1, 11, 64), ("L3 3x3 dgrad up_conv3", 56, 256, 1, 11, 512),
          ("L3 3x3 dgrad down3", 56, 256, 1, 11, 128), ("L3 3x3 fwd down3", 56, 128, 1, 9, 256)]
