#!/bin/bash
# tools/ab_post_zinit.sh -- on the GPU box: config 5 (2000 mixed families, vcf_mode) with lean_nuc_post's kid sums
# starting from their first term (default) against the former 0.0 start (lib_exp/zinit0.so, PM_POST_ZINIT=0)
set -e
B="python3 bench.py --no-cpu-baseline --shape mixed --families 2000 --vcf --no-denovo --batch 65536 --steps 60"
O=gpurun_out/ab_post_zinit.txt
: > $O
for rep in 1 2 3; do
  for lib in polymutt_amd/lib_exp/zinit0.so ""; do
    echo "rep $rep lib=${lib:-default}" >> $O
    POLYMUTT_LIB=$lib timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4),'ms')" >> $O
  done
done
cat $O
