set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/tr
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/gpu_tests.log 2>&1 || { tail -30 $R/gpurun_out/gpu_tests.log; exit 1; }
tail -2 $R/gpurun_out/gpu_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr/q -o run -- python3 $R/bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-denovo > $R/gpurun_out/tr/q.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr/dn -o run -- python3 $R/bench.py --steps 10 --warmup 1 --denovo --no-cpu-baseline > $R/gpurun_out/tr/dn.log 2>&1 || exit 1
