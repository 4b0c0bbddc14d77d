#!/bin/bash
# Round 5: the driver-style bench line (--steps 20 --warmup 5) and rocprofv3 kernel-trace of the identical
# command, summarised over the timed window and its traced re-run (tools/kernel_window.py).
# usage: bash tools/r05_window.sh [model] [steps] [warmup] [extra bench args...]
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
M=${1:-humanoid}; K=${2:-20}; W=${3:-5}; shift 3 2>/dev/null
tag=${M}_s${K}${TAG:+_$TAG}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --model $M --steps $K --warmup $W --cpu-baseline 0 "$@" > gpurun_out/bench_$tag.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$tag.log | cut -c1-400
d=gpurun_out/win_$tag
rm -rf $d
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --model $M --steps $K --warmup $W --cpu-baseline 0 "$@" > $d.log 2>&1 || exit $?
python3 tools/kernel_window.py $d $W $K gpurun_out/window_$tag.json > /dev/null || exit $?
python3 - "$tag" <<'PY'
import json, sys
tag = sys.argv[1]
w = json.load(open(f"gpurun_out/window_{tag}.json"))
b = json.loads([l for l in open(f"gpurun_out/win_{tag}.log") if l.startswith("{")][-1])
r = b["roofline"]
print(tag, "bench(rocprof run) ms/step", round(b["ms_per_step"], 4), "trace sum", round(b["config"]["trace_kernel_sum_ms_per_step"], 4),
      "dominant", r["group"], round(r["kernel_ms"], 4), "frac", round(r["frac"], 4))
for wn in ("timed", "trace"):
  x = w[wn]
  print(" rocprof", wn, "steps", x["steps"], "sum", round(x["kernel_sum_ms_per_step"], 4), "span", x["span_ms_per_step"] and round(x["span_ms_per_step"], 4),
        {k.split("::")[-1][:40]: round(v["ms_per_step"], 4) for k, v in x["kernels"].items()})
print(" bench kernels", {k.split("::")[-1][:40]: round(v["ms_per_step"], 4) for k, v in r["kernels"].items()})
PY
