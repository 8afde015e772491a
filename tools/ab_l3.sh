mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_corpus.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/ab_tests.log; exit 1; }
for G in 4 2; do FHEICP_V4_G=$G timeout -k 10 100 python tools/prof_br.py --variants 4 --rounds 2 --P 21 2>&1 | grep -v amdgpu.ids | sed "s/^/P21 G=$G /" || exit 1; done
FHEICP_V4_G=4 timeout -k 10 100 python tools/prof_br.py --variants 4 --rounds 2 --P 16 2>&1 | grep -v amdgpu.ids | sed "s/^/P16 G=4 /"
