# GPU check of the exact 32-bit accumulator rounding: noise and time per gadget, 64-bit comparison, all GPU tests, the headline bench
mkdir -p gpurun_out
GADGETS="15,2 23,1 22,1 21,1" bash tools/ab_gadgets.sh > gpurun_out/ab_gadgets2.log 2>&1 || { cat gpurun_out/ab_gadgets2.log; exit 1; }
FHEICP_V4_G=2 FHEICP_V4_A64=1 timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 2 --P 16 >> gpurun_out/ab_gadgets2.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/ab_gadgets2.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cut -c1-300 gpurun_out/bench.json
