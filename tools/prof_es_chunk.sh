#!/bin/bash
# tools/prof_es_chunk.sh -- on the GPU box: kernel-trace stats of config 4 BA (one engine) at the former 65 532-item
# chunk (PM_ES_CHUNK=65532) and at the default (a whole batch per chunk)
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT}
B="$R/bench.py --no-cpu-baseline --engines 1 --shape ext10 --families 200 --no-denovo --batch 16384 --steps 8 --warmup 2 --calib-steps 0"
PM_ES_CHUNK=65532 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pch_old -o run -- python3 $B > $R/gpurun_out/pch_old.json 2>/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pch_new -o run -- python3 $B > $R/gpurun_out/pch_new.json 2>/dev/null
