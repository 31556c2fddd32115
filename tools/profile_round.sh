#!/bin/bash
# tools/profile_round.sh ROUND -- run on the GPU box (via gpurun) to collect the round's profiles:
#   1. rocprofv3 --kernel-trace --stats of the default bench command (kernel time summary)
#   2. separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ busy/stall counters) -- never combined with
#      any other trace domain
#   3. the FP64 issue-rate microbenchmark (tools/fp64_peak)
# Outputs land in gpurun_out/prof_$ROUND/; tools/summarize_profile.py turns them into profiles/.
set -u
ROUND=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$ROUND
mkdir -p "$OUT"
echo "revision: $(cat "$R/REVISION" 2>/dev/null || echo unknown)" > "$OUT/revision.txt"
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --no-cpu-baseline --steps 40 --calib-steps 4"
ONLY=${PR_ONLY:-}   # PR_ONLY="a b c": run only these steps (a round's passes split over several gpurun calls)
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $name "* ]]; then return 0; fi
  echo "[$(date +%T)] $name" >&2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc" >&2; tail -20 "$OUT/$name.err" >&2; exit $rc; fi
}
step fp64_peak 120 "$R/tools/fp64_peak"
# the default bench line itself (with its cpu_baseline leg), as the driver runs it
step bench 600 python3 $R/bench.py
# default bench (3 overlapping engines): whole-step kernel mix; per-kernel durations there include GPU sharing
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $BENCH
# one engine: each kernel alone on the GPU -- the per-kernel times the roofline uses
step trace1 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace1" -o run -- $BENCH --engines 1
# BASELINE config 4 shape (200 ext10 pedigrees, Elston-Stewart peeling), one engine
step trace_ext10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_ext10" -o run -- $BENCH --engines 1 --shape ext10 --families 200 --batch 16384 --no-denovo --steps 8
step trace_ext10dn 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_ext10dn" -o run -- $BENCH --engines 1 --shape ext10 --families 200 --batch 4096 --steps 6
# BASELINE config 5 shape (2000 mixed families, --in_vcf engine mode), one engine
step trace_cfg5 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_cfg5" -o run -- $BENCH --engines 1 --shape mixed --families 2000 --vcf --no-denovo --batch 65536 --steps 12
step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- $BENCH --engines 1 --steps 4 --warmup 1 --calib-steps 0
step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- $BENCH --engines 1 --steps 4 --warmup 1 --calib-steps 0
step pmc_sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/pmc_sq" -o run -- $BENCH --engines 1 --steps 4 --warmup 1 --calib-steps 0
step pmc_sq2 400 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_INSTS_SMEM --output-format csv -d "$OUT/pmc_sq2" -o run -- $BENCH --engines 1 --steps 4 --warmup 1 --calib-steps 0
step pmc_sq3 400 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_sq3" -o run -- $BENCH --engines 1 --steps 4 --warmup 1 --calib-steps 0
# config 4 BA's EP k_brent and hoisting kernels: SQ and FETCH passes (one engine)
E10="$BENCH --engines 1 --shape ext10 --families 200 --batch 16384 --no-denovo --steps 4 --warmup 1 --calib-steps 0"
step pmc_ext10_sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/pmc_ext10_sq" -o run -- $E10
step pmc_ext10_sq2 400 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_INSTS_SMEM --output-format csv -d "$OUT/pmc_ext10_sq2" -o run -- $E10
step pmc_ext10_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_ext10_fetch" -o run -- $E10
# config 4 --denovo's hoisting (es_hoist_wave) and config 5's kernels: SQ and FETCH passes (one engine)
E10D="$BENCH --engines 1 --shape ext10 --families 200 --batch 4096 --steps 4 --warmup 1 --calib-steps 0"
step pmc_ext10dn_sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/pmc_ext10dn_sq" -o run -- $E10D
step pmc_ext10dn_sq2 400 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_INSTS_SMEM --output-format csv -d "$OUT/pmc_ext10dn_sq2" -o run -- $E10D
step pmc_ext10dn_sq3 400 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_ext10dn_sq3" -o run -- $E10D
C5="$BENCH --engines 1 --shape mixed --families 2000 --vcf --no-denovo --batch 65536 --steps 4 --warmup 1 --calib-steps 0"
step pmc_cfg5_sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/pmc_cfg5_sq" -o run -- $C5
step pmc_cfg5_sq2 400 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_INSTS_SMEM --output-format csv -d "$OUT/pmc_cfg5_sq2" -o run -- $C5
step pmc_cfg5_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_cfg5_fetch" -o run -- $C5
# config 4 at its 8-12-member range (extmix), one engine
step trace_extmix 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_extmix" -o run -- $BENCH --engines 1 --shape extmix --families 200 --batch 16384 --no-denovo --steps 8
# the other BASELINE configs' bench lines (default three engines)
B="python3 $R/bench.py --no-cpu-baseline"
step cfg2 300 $B --shape trio --families 1000 --no-denovo --steps 100
step cfg4 300 $B --shape ext10 --families 200 --no-denovo --batch 16384 --steps 30
step cfg4dn 300 $B --shape ext10 --families 200 --batch 4096 --steps 20
step cfg4mix 300 $B --shape extmix --families 200 --no-denovo --batch 16384 --steps 30
step cfg4mixdn 300 $B --shape extmix --families 200 --batch 4096 --steps 20
step cfg5 300 $B --shape mixed --families 2000 --vcf --no-denovo --batch 65536 --steps 60
step cfg3plain 300 $B --no-denovo --steps 200
echo done >&2
