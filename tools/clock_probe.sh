mkdir -p gpurun_out
timeout -k 10 100 python tools/prof_br.py --variants 4 --rounds 2 --stamps > gpurun_out/stamps2.txt 2>&1 || exit 1
(timeout -k 10 120 python tools/prof_br.py --variants 4 --rounds 40 > gpurun_out/long.txt 2>&1 &)
sleep 25; rocm-smi --showclocks --showpower --showtemp > gpurun_out/smi1.txt 2>&1; sleep 3; rocm-smi --showclocks --showpower > gpurun_out/smi2.txt 2>&1
wait; sleep 20; cat gpurun_out/long.txt | tail -2
