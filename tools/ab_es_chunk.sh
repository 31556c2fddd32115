#!/bin/bash
# tools/ab_es_chunk.sh -- on the GPU box: config 4 BA (200 ext10, 16 384-site batches) and --denovo (4 096-site
# batches) with the coefficient chunk covering a whole batch's items (default) against the former chunk 4 items
# short of it (PM_ES_CHUNK=65532 / 16380: an empty second chunk per list, one extra hoisting + Brent launch pair).
set -e
B="python3 bench.py --no-cpu-baseline --shape ext10 --families 200"
O=gpurun_out/ab_es_chunk.txt
: > $O
for rep in 1 2; do
  for cfg in "65532|--no-denovo --batch 16384 --steps 30" "16380|--batch 4096 --steps 20"; do
    old=${cfg%%|*}; args=${cfg#*|}
    for ch in $old ""; do
      echo "rep $rep PM_ES_CHUNK=${ch:-default} $args" >> $O
      PM_ES_CHUNK=$ch timeout -k 10 200 $B $args 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4),'ms k_brent frac', round(d['roofline']['frac'],4), 'hoist ms', round(d['roofline_es_hoist']['avg_launch_ms'],4), 'frac', round(d['roofline_es_hoist']['frac'],4))" >> $O
    done
  done
done
cat $O
