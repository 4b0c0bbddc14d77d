cd $GRAFT_REPO_ROOT
for pad in 0 2300 6100 12000; do
  MJW_LDS_PAD=$pad timeout -k 10 200 python bench.py --steps 200 --cpu-baseline 0 > gpurun_out/occ_$pad.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/occ_$pad.log').read().strip().splitlines()[-1]); print($pad, round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4))"
done
