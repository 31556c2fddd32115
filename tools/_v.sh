set -o pipefail
mkdir -p gpurun_out/v3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
B="timeout -k 10 150 python -u bench.py --steps 30 --warmup 2 --no-cpu-baseline"
for v in 16 8 4 1; do PM_PREP_VEC=$v $B --no-denovo > gpurun_out/v3/q$v.log 2>&1 || exit 1; PM_PREP_VEC=$v $B > gpurun_out/v3/dn$v.log 2>&1 || exit 1; done
