# round-5 GPU call 2: planner calibration, full GPU suite, bench, GEMM probe incl. square shapes
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_memory_gpu.py -q -s --timeout 240 --timeout-method thread > gpurun_out/mem2.log 2>&1
echo "mem rc=$?"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_memory_gpu.py > gpurun_out/t2.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b2.log 2>&1 || exit $?
timeout -k 10 400 python tools/gemm4_probe.py --layouts nt tn --shapes gateup lmhead qkv sq4k sq8k --big --scheds 1 --rounds 5 --iters 5 > gpurun_out/probe2.log 2>&1
echo "probe rc=$?"
tail -3 gpurun_out/t2.log; tail -1 gpurun_out/b2.log
