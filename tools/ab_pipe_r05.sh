set -u -o pipefail
mkdir -p gpurun_out/r05g
for rep in 1 2; do
  for pm in 2048 1024; do
    FHEICP_PIPE_MIN=$pm timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r05g/c2_pm${pm}_$rep.json 2> gpurun_out/r05g/c2_pm${pm}_$rep.err || exit 1
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --docs 12500 --steps 2 --warmup 1 > gpurun_out/r05g/c4.json 2> gpurun_out/r05g/c4.err || exit 1
