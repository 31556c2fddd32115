#!/bin/bash
# tools/cli_e2e.sh NFAM NSITES [IO_THREADS...] -- end-to-end CLI timing (GLF ingest + engine + VCF) on a
# synthetic dataset: the product binary (once per --io_threads value; default: its own default) vs the
# reference harness (oracle/_ref/pm_ref, 8 threads; skipped with SKIP_REF=1), same inputs.  One JSON line.
set -eu
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
NF=${1:-1000}; NS=${2:-2000}; shift 2 || true
IOS=${*:-0}
D=$(mktemp -d /tmp/pm_e2e.XXXX)
trap 'rm -rf "$D"' EXIT
python3 -c "import sys; sys.path.insert(0, '$R'); import polymutt_amd as pm; pm.synth_write_dataset('$D', 'quad', $NF, $NS, 7)"
cd "$D"
GPU=""
for io in $IOS; do
  t0=$(date +%s.%N)
  PM_TIMING=1 timeout -k 10 600 "$R/polymutt_amd/bin/polymutt" -p test.ped -d test.dat -g test.gif --out_vcf gpu.vcf --io_threads $io > gpu.log 2> gpu_$io.err; cat gpu_$io.err >&2
  t1=$(date +%s.%N)
  GPU="$GPU\"io_threads_$io\": $(python3 -c "print(round($t1 - $t0, 3))"), "
done
REF=""
if [ -x "$R/oracle/_ref/pm_ref" ] && [ "${SKIP_REF:-0}" != 1 ]; then
  t1=$(date +%s.%N)
  timeout -k 10 900 "$R/oracle/_ref/pm_ref" -p test.ped -d test.dat -g test.gif --out_vcf ref.vcf --nthreads 8 > ref.log
  t2=$(date +%s.%N)
  same=$(diff <(grep -v '^##' gpu.vcf) <(grep -v '^##' ref.vcf) > /dev/null && echo true || echo false)
  REF=", \"reference_s\": $(python3 -c "print(round($t2 - $t1, 3))"), \"vcf_identical\": $same"
fi
echo "{\"families\": $NF, \"sites\": $NS, \"gpu_cli_s\": {${GPU%, }}$REF, \"glf_bytes\": $(du -sb . | cut -f1)}"
