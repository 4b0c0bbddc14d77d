set -e
C="--steps 5 --warmup 2 --cpu-baseline 0 --nworld 301"
timeout -k 10 120 python bench.py --gpus 1 $C --dump-qpos gpurun_out/p_eager > /dev/null
timeout -k 10 120 python bench.py --gpus 1 --graph 1 $C --dump-qpos gpurun_out/p_graph > /dev/null
timeout -k 10 120 python bench.py --gpus 2 --scaling strong $C --dump-qpos gpurun_out/p_strong > /dev/null
timeout -k 10 120 python bench.py --gpus 1 --nworld 151 --steps 5 --warmup 2 --cpu-baseline 0 --dump-qpos gpurun_out/p_151 > /dev/null
python - <<'PY'
import numpy as np
L=lambda p: np.load(p)["qpos"]
e=L("gpurun_out/p_eager/qpos_rank0.npz"); g=L("gpurun_out/p_graph/qpos_rank0.npz")
s0=L("gpurun_out/p_strong/qpos_rank0.npz"); s1=L("gpurun_out/p_strong/qpos_rank1.npz"); o=L("gpurun_out/p_151/qpos_rank0.npz")
print("eager vs graph", abs(e-g).max())
print("eager vs strong", abs(e-np.concatenate([s0,s1])).max(), s0.shape, s1.shape)
print("eager[:151] vs 151-run", abs(e[:151]-o).max(), "strong0 vs 151-run", abs(s0-o).max())
PY
