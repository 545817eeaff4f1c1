#!/usr/bin/env python3
"""Export the reference's MatNet weights (NetWeights/{Intel,Amd,P100}_weights.h5,
loaded by IA-SPGEMM-CPU_release/MatNet.py:81 and IA-SPGEMM-GPU_release/MatNet.py:78)
to the flat blobs libias.so's selector reads: ia-spgemm_amd/data/matnet_<name>.bin.

Runs in the build container only (it reads /root/reference); the blobs are
committed, so the GPU box never needs the reference.  The .h5 files are read
with tools/h5min.py, which executes nothing from them.

Blob layout (little-endian): magic "IASMNET1", int32 nfeatures, int32
nclasses, then float32 arrays in Keras layouts, in this order:
  conv2d_1..3 (image branch 1: 3x3x1x16 valid, 5x5x16x16 s2 same, 5x5x16x16 s2 same),
  conv2d_4..6 (image branch 2, same shapes), each kernel then bias;
  dense_1 (features: nf x nf), dense_2 / dense_3 (images: 256 x 32),
  dense_4 (output: (64 + nf) x nclasses), each kernel then bias.
Layer names follow the construction order in MatNet.py Pred() (CPU :45-77).
"""
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from h5min import H5  # noqa: E402

ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "ia-spgemm_amd", "data")
REF = "/root/reference/NetWeights"
SETS = {"intel": "Intel_weights.h5", "amd": "Amd_weights.h5", "p100": "P100_weights.h5"}
ORDER = ["conv2d_1", "conv2d_2", "conv2d_3", "conv2d_4", "conv2d_5", "conv2d_6",
         "dense_1", "dense_2", "dense_3", "dense_4"]


def arrays(src):
    """{layer: (kernel, bias)} of one weight file, float32."""
    a = dict(H5(src).walk())
    return {l: (np.asarray(a[f"/{l}/{l}/kernel:0"], "<f4"), np.asarray(a[f"/{l}/{l}/bias:0"], "<f4"))
            for l in ORDER}


def export(name, src, dst):
    w = arrays(src)
    nf = w["dense_1"][0].shape[0]
    nc = w["dense_4"][0].shape[1]
    with open(dst, "wb") as f:
        f.write(b"IASMNET1")
        f.write(struct.pack("<ii", nf, nc))
        for layer in ORDER:
            for a in w[layer]:
                f.write(np.ascontiguousarray(a).tobytes())
    print(f"{name}: {src} -> {dst} (features {nf}, classes {nc})")


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, fn in SETS.items():
        export(name, os.path.join(REF, fn), os.path.join(OUT, f"matnet_{name}.bin"))


if __name__ == "__main__":
    main()
