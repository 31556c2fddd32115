#!/bin/bash
# tools/cli_e2e.sh NFAM NSITES -- end-to-end CLI timing (GLF ingest + engine + VCF) on a synthetic dataset,
# product binary vs the reference harness (oracle/_ref/pm_ref), same inputs.  Prints one JSON line.
set -eu
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
NF=${1:-1000}; NS=${2:-2000}
D=$(mktemp -d /tmp/pm_e2e.XXXX)
python3 -c "import sys; sys.path.insert(0, '$R'); import polymutt_amd as pm; pm.synth_write_dataset('$D', 'quad', $NF, $NS, 7)"
cd "$D"
t0=$(date +%s.%N)
timeout -k 10 600 "$R/polymutt_amd/bin/polymutt" -p test.ped -d test.dat -g test.gif --out_vcf gpu.vcf > gpu.log
t1=$(date +%s.%N)
REF=""
if [ -x "$R/oracle/_ref/pm_ref" ]; then
  timeout -k 10 900 "$R/oracle/_ref/pm_ref" -p test.ped -d test.dat -g test.gif --out_vcf ref.vcf --nthreads 8 > ref.log
  t2=$(date +%s.%N)
  same=$(diff <(grep -v '^##' gpu.vcf) <(grep -v '^##' ref.vcf) > /dev/null && echo true || echo false)
  REF=", \"reference_s\": $(python3 -c "print($t2 - $t1)"), \"vcf_identical\": $same"
fi
echo "{\"families\": $NF, \"sites\": $NS, \"gpu_cli_s\": $(python3 -c "print($t1 - $t0)")$REF}"
rm -rf "$D"
