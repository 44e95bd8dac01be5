#!/usr/bin/env python3
"""Diagnostic (GPU): a default-C5-like world match launch in the accept-only form, 125 problems x
2,000 queries x 5,000 random references, five times (for PMC passes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "02-visualodometry_amd"))


def main():
    import numpy as np
    import picp_amd
    rng = np.random.default_rng(1)
    dq = [rng.uniform(-1, 1, (2000, 10)).astype(np.float32) for _ in range(125)]
    dr = [rng.uniform(-1, 1, (5000, 10)).astype(np.float32) for _ in range(125)]
    for _ in range(5):
        picp_amd.match_points_batch(dq, dr, 0.2, 0.8, form="accept_only")
    print("ok")


if __name__ == "__main__":
    main()
