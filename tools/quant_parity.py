"""Input quantiser contract vs the float readings of MnistUtils.cpp:83-93, at every BASELINE shape.

The device quantiser (csrc/niti_quant.hip) and its oracle O.quantize_images use exact integer
statistics of the uint8 pixels.  The reference computes the same expression in float, its two full
reductions summed in an order the source does not fix under -ffast-math (CMakeLists.txt:429-430):
the C loop is sequential (CPUReduction.cpp:86-95), a vectorising compiler may run it in 4 / 8 / 16
interleaved lanes.  For each shape and order this prints how many int8 inputs and whether ascale
differ from the exact-statistics contract.  Seeded uniform uint8 images (the bench's input).

    python tools/quant_parity.py [--big]      (--big adds the 8-GPU global batches: 512 / 1024 x 224 px)
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import niti_oracle as O  # noqa: E402

SHAPES = [
    ("cfg 1/2 LeNet MNIST batch 64", (64, 1, 28, 28)),
    ("cfg 3 VGG-11 CIFAR batch 256", (256, 3, 32, 32)),
    ("cfg 4 VGG-16 224 px, 64 per GPU", (64, 3, 224, 224)),
    ("cfg 5 ResNet-18 224 px, 128 per GPU", (128, 3, 224, 224)),
]
BIG = [
    ("cfg 4 VGG-16 global batch 512", (512, 3, 224, 224)),
    ("cfg 5 ResNet-18 global batch 1024", (1024, 3, 224, 224)),
]
LANES = (1, 4, 8, 16)


def count(shape, seed=1):
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, shape, dtype=np.uint8)
    x, a = O.quantize_images(img)
    f = img.astype(np.float32)
    res = []
    for lanes in LANES:
        xf, af = O.quantize_input(f, lanes)
        d = np.abs(x.astype(np.int16) - xf.astype(np.int16))
        # the quantiser maps each of the 256 pixel values to one int8 code: count the values whose
        # code differs (every pixel of such a value flips)
        classes = int(np.unique(img[d > 0]).size)
        res.append((lanes, int((d > 0).sum()), int(d.max()), a == af, classes))
        del xf
    return img.size, a, res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--seeds", default="1,5")
    args = ap.parse_args()
    print("uniform uint8 images (np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8));")
    print("exact-statistics contract (device, O.quantize_images) vs the float reading with its two sums in")
    print("`lanes` interleaved partials (1 = the C loop's sequential order).  Cell: differing int8 inputs /")
    print("pixel-value classes of 256 whose code differs, max |difference|, ascale equal (y / N)")
    print(f"{'seed':>4} {'shape':<16} {'inputs':>10} ascale " + "".join(f"{'lanes=' + str(l):>25}" for l in LANES))
    for seed in [int(v) for v in args.seeds.split(",")]:
        for name, shape in SHAPES + (BIG if args.big else []):
            t = time.time()
            n, a, res = count(shape, seed)
            cells = "".join(f"{f'{c} / {k} ({m}, {chr(121) if eq else chr(78)})':>25}" for _, c, m, eq, k in res)
            print(f"{seed:>4} {'x'.join(map(str, shape)):<16} {n:>10} {a:>6} {cells}   [{name}, {time.time() - t:.1f} s]")


if __name__ == "__main__":
    main()
