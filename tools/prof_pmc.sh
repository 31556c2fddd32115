#!/bin/bash
# tools/prof_pmc.sh TAG BENCH_ARGS... -- on the GPU box (via gpurun): SQ instruction-mix / stall PMC passes and the HBM
# FETCH pass of one bench configuration on one engine, each pass its own run (rocprofv3 does not split counters).
# POLYMUTT_LIB in the environment selects a library variant.  Outputs: gpurun_out/pmc_TAG/<pass>/run_counter_collection.csv
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
echo "revision: $(cat "$R/REVISION" 2>/dev/null || echo unknown) lib: ${POLYMUTT_LIB:-default}" > "$OUT/revision.txt"
B="python3 $R/bench.py --no-cpu-baseline --engines 1 $* --steps 2 --warmup 1 --calib-steps 0"
pass() {   # pass NAME COUNTERS...
  local name=$1; shift
  echo "[$(date +%T)] $name" >&2
  timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- $B > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "pass $name failed rc=$rc" >&2; tail -20 "$OUT/$name.err" >&2; exit $rc; fi
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD
pass sq2 SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA
pass sq3 SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
echo done >&2
