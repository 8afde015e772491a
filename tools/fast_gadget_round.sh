# GPU check of the per-round gadget change: its parity tests, then the C3, C5 and corpus benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "fast or sign_real or keygen or sign_toy" > gpurun_out/fast_tests.log 2>&1 || { tail -30 gpurun_out/fast_tests.log; exit 1; }
tail -3 gpurun_out/fast_tests.log
timeout -k 10 400 python bench.py --docs 10000 --dim 32 --n-bits 8 --steps 2 > gpurun_out/c3.json 2> gpurun_out/c3.err || exit 1
timeout -k 10 400 python bench.py --docs 1000 --dim 768 --n-bits 8 --steps 2 > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
timeout -k 10 400 python bench.py --mode corpus --steps 2 > gpurun_out/corpus.json 2> gpurun_out/corpus.err || exit 1
cut -c1-400 gpurun_out/c3.json gpurun_out/c5.json gpurun_out/corpus.json
