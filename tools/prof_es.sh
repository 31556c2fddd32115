#!/bin/bash
# tools/prof_es.sh TAG -- run on the GPU box (via gpurun): where k_brent's time goes, per BASELINE shape.
#   1. in-kernel hoisting / evaluation split (PM_PHASE_TIMING=1) of the one-engine bench for 200 ext10 pedigrees
#      (plain and --denovo) and 1000 quads --denovo
#   2. PMC passes (SQ instruction mix and stall split, HBM FETCH) of the ext10 plain bench, each its own run
#   3. rocprofv3 -L (the counter names this box offers)
# Outputs: gpurun_out/prof_TAG/*.out|*.err and the rocprofv3 directories.
set -u
TAG=${1:-es}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
echo "revision: $(cat "$R/REVISION" 2>/dev/null || echo unknown)" > "$OUT/revision.txt"
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name" >&2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc" >&2; tail -20 "$OUT/$name.err" >&2; exit $rc; fi
}
B="python3 $R/bench.py --no-cpu-baseline --engines 1"
EXT="$B --shape ext10 --families 200 --no-denovo --batch 16384 --steps 8 --calib-steps 4"
EXTDN="$B --shape ext10 --families 200 --batch 4096 --steps 6 --calib-steps 3"
QDN="$B --steps 12 --calib-steps 4"
export PM_PHASE_TIMING=1
step phase_ext10 300 $EXT
step phase_ext10dn 300 $EXTDN
step phase_quad_dn 300 $QDN
unset PM_PHASE_TIMING
step list 120 rocprofv3 -L
step trace_ext10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_ext10" -o run -- $EXT
step pmc_sq1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/pmc_sq1" -o run -- $EXT --steps 2 --warmup 1 --calib-steps 0
step pmc_sq2 300 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA --output-format csv -d "$OUT/pmc_sq2" -o run -- $EXT --steps 2 --warmup 1 --calib-steps 0
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- $EXT --steps 2 --warmup 1 --calib-steps 0
echo done >&2
