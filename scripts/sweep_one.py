#!/usr/bin/env python3
"""One fused-sweep case (default: 2^24 c64 tensor, 4 gates on the innermost legs), run a few
times — a small target for rocprofv3 --pmc passes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sweep_bench import case
n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
case(n, [(n - 1, n - 2), (n - 3, n - 4), (n - 2, n - 3), (n - 1, n - 4)], reps=5)
