set -e
for args in "--steps 20 --warmup 5" "--steps 20 --warmup 5" "--steps 20 --warmup 60" "--steps 100 --warmup 5"; do
  timeout -k 10 200 python -u bench.py --cpu-baseline 0 $args > gpurun_out/probe.json 2> gpurun_out/probe.err
  python - "$args" <<'PY'
import json,sys
l=[x for x in open('gpurun_out/probe.json') if x.startswith('{')][-1]
d=json.loads(l)
t=d.get('timing') or {}
print(sys.argv[1], 'ms/step', round(d['ms_per_step'],4), 'value', round(d['value']/1e6,3), {k:v for k,v in d.items() if k in ('trace_sum_ms_per_step','window')}, str(t)[:400], flush=True)
PY
done
