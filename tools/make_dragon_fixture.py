#!/usr/bin/env python3
"""Writes tests/golden/dragon10k_tris.npy: the 9,992 triangles of the reference's
examples/practice5_dragon_10k.txt (TRIANGLE x0 y0 z0 x1 y1 z1 x2 y2 z2 lines) as float32
(n, 3, 3).  Data only (vertex positions), for the C5 proxy scene (scenes.make_sponza_dragon,
SURVEY.md §8 C5 and §7 "a dragon_100k proxy (1->4 subdivision of the 10k dragon)").
Run here, where /root/reference exists; the GPU box uses the committed .npy."""
import os
import sys

import numpy as np

SRC = "/root/reference/examples/practice5_dragon_10k.txt"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden", "dragon10k_tris.npy")


def main():
    tris = []
    with open(sys.argv[1] if len(sys.argv) > 1 else SRC) as f:
        for line in f:
            if line.startswith("TRIANGLE "):
                v = [float(x) for x in line.split()[1:]]
                assert len(v) == 9, line
                tris.append(v)
    a = np.asarray(tris, np.float32).reshape(-1, 3, 3)
    np.save(OUT, a)
    print(OUT, a.shape)


if __name__ == "__main__":
    main()
