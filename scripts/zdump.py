#!/usr/bin/env python3
"""Debug helper: compress segments on the GPU and save the frames (gpurun_out/zdump.npz)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bitar_amd
import oracle_lib as O
kind, seg = int(sys.argv[1]), int(sys.argv[2])
n = 5 * seg + seg // 3 + 1
data = O.fill(kind, 77, n)
eng = bitar_amd.Engine(0)
d = torch.from_numpy(data).cuda()
slab, stride, sizes = eng.compress(bitar_amd.CODEC_ZSTD, d, seg)
eng.sync()
np.savez("gpurun_out/zdump.npz", slab=slab.cpu().numpy(), sizes=sizes.cpu().numpy(), stride=stride)
print("saved", sizes.cpu().numpy())
