# light-stamp profile with the raw per-wave stamps dumped (H12_WAVE_DUMP) for the distribution of wave durations
set -o pipefail
tag=${1:-r5}
H12_PHASE_LIGHT=1 H12_WAVE_DUMP=gpurun_out/${tag}_waves.npy timeout -k 10 200 python3 -u tools/phase_profile.py --tag light $EXTRA > gpurun_out/${tag}_light.json 2>/dev/null || { echo "light failed"; exit 1; }
python3 - $tag <<'PY'
import sys, numpy as np, json
tag = sys.argv[1]
R = np.load(f"gpurun_out/{tag}_waves.npy")  # (launches, waves, 7): start, end, end+wait, after physics, after reset, xcc, after F
rs = np.load(f"gpurun_out/{tag}_waves_resets.npy")
phys = (R[:, :, 3] - R[:, :, 0]) / 100.0
dur = (R[:, :, 1] - R[:, :, 0]) / 100.0
post = (R[:, :, 1] - R[:, :, 3]) / 100.0
start = (R[:, :, 0] - R[:, :, 0].min(1, keepdims=True)) / 100.0
end = (R[:, :, 2] - R[:, :, 0].min(1, keepdims=True)) / 100.0
q = lambda x: [round(float(np.quantile(x, p)), 2) for p in (0.05, 0.5, 0.95, 1.0)]
print("physics loop us p5/p50/p95/max", q(phys))
print("post-loop us", q(post))
print("wave duration us", q(dur))
print("start offset us", q(start))
print("end offset us", q(end))
# which wave is last in each launch, and why
last = end.argmax(1)
print("last wave: physics loop", [round(float(phys[i, w]), 2) for i, w in enumerate(last)][:10])
print("last wave: start offset", [round(float(start[i, w]), 2) for i, w in enumerate(last)][:10])
print("last wave: resets", [int(rs[i, w]) for i, w in enumerate(last)][:10])
print("corr(phys, resets)", round(float(np.corrcoef(phys.ravel(), rs.ravel())[0, 1]), 3))
x = R[:, :, 5].ravel(); p = phys.ravel()
print("physics p50 per xcc", {int(c): round(float(np.median(p[x == c])), 2) for c in np.unique(x)})
PY
