set -e
B="python3 bench.py --no-cpu-baseline"
O=gpurun_out/ab_spw.txt
: > $O
for spw in 8 ""; do
  for cfg in "--shape ext10 --families 200 --no-denovo --batch 16384 --steps 30" "--shape ext10 --families 200 --batch 4096 --steps 20" "--shape mixed --families 2000 --vcf --no-denovo --batch 65536 --steps 60"; do
    echo "PM_PREP_SPW=${spw:-auto} $cfg" >> $O
    PM_PREP_SPW=$spw timeout -k 10 200 $B $cfg 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4),'ms')" >> $O
  done
done
cat $O
