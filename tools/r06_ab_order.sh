#!/bin/bash
# A/B of the longest-first world order (MJW_WORLD_ORDER=0 turns it off) on the dense-path benches, same box:
# humanoid CG (driver window and 300 steps), humanoid / franka / apollo Newton (300 steps), then the Newton
# phase split with the order off.  usage: bash tools/r06_ab_order.sh [noprof]
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
line() {
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(round(d['value']/1e6,3),'M', round(d['ms_per_step'],4), {k.split('<')[0].split('::')[-1]+('<'+k.split('<')[1][:12] if '<' in k else ''): round(v['ms_per_step'],4) for k,v in d['roofline']['kernels'].items()})" "$1"
}
for rep in 1 2; do
  for args in "--steps 20 --warmup 5" "--steps 300 --warmup 20" "--steps 300 --warmup 20 --solver NEWTON" "--model franka --steps 300 --warmup 20" "--model apollo --steps 300 --warmup 20"; do
    for ord in 1 0; do
      MJW_WORLD_ORDER=$ord timeout -k 10 300 python -u bench.py $args --cpu-baseline 0 > gpurun_out/ab_order.log 2>&1 || { tail -3 gpurun_out/ab_order.log; exit 1; }
      echo "rep $rep order=$ord [$args]: $(line gpurun_out/ab_order.log)"
    done
  done
done
if [ "$1" != "noprof" ]; then
  MJW_WORLD_ORDER=0 timeout -k 10 300 python -u tools/phase_prof.py 8192 20 NEWTON humanoid 5 > gpurun_out/r06_phase_newton_noorder.log 2>&1 || { tail -5 gpurun_out/r06_phase_newton_noorder.log; exit 1; }
  cat gpurun_out/r06_phase_newton_noorder.log
fi
exit 0
