"""Fusion and batching switches of the HIP front end (ops/hip*.py), in one place so a GPU test can
compare each fused path against the unfused composition it replaces (production keeps them on).
Read at call time (``fusion.BNB``), so flipping one affects every module that honours it."""

G2_GROUP = True      # strided dgrad phases in one launch (ops/hip.py conv2d_dgrad)
BNB = True           # backward-BatchNorm fusion (ReLU mask + statistics) into the producing dgrad /
                     # max-pool backward epilogue, and BatchNorm + ReLU + max-pool in one forward pass
BN_DUAL = True       # projection-shortcut BatchNorm pairs in one pass (forward apply, backward)
DEFER_REDUCE = True  # one batched split-K weight-gradient reduce per backward
HWGRAD_S2 = True     # 3x3 stride-2 weight gradients on the stride-2 halo kernel (else gemm_t2)
HCONV_1X1 = True     # 1x1 convs on the halo kernel (else the routing table's GEMM choice; test hook)
