#!/bin/bash
# The other BASELINE configs on one GPU (profiles/r01_c*_bench.json).
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --docs 10000 --dim 32 --n-bits 8 --steps 2 > gpurun_out/c3.json 2> gpurun_out/c3.err || exit 1
timeout -k 10 300 python bench.py --docs 12500 --dim 16 --n-bits 6 --steps 2 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 1
timeout -k 10 400 python bench.py --docs 1000 --dim 768 --n-bits 8 --steps 2 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
