#!/usr/bin/env python3
"""Gates of the sole-contact scenarios (tests/test_gpu_sensitivity.py::test_forced_sole_contact_scenarios) from the
kernel's measured floors: profiles/r5/bias_<scenario>[_rsl].json, written by that test under H12_GATE_MEASURE=<dir>
on the GPU (the per-field mean / standard error of the signed relative error over the passing env-steps, and the
absolute-error quantiles).  Writes tests/golden/sole_bias_gate.json:

  bias[key][field] = 3 |mean| + 6 max(se, se_cpu) + 1e-9
                     (the kernel's own fp32 bias, x3, plus 6 standard errors of the mean: the larger of the kernel's
                     and that of tests/test_forced_harness.py's clean CPU stand-in, whose rounding noise is calibrated
                     to the kernel's floor, so the harness's clean run and the kernel pass by the same margin)
  quant[key][crit] = (2 p50, 2 p99)           (the absolute-error quantiles, x2)

    python tools/gen_sole_bias_gate.py [profiles/r5]
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main():
    src = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "profiles" / "r5"
    out = {"source": str(src.relative_to(ROOT)) if src.is_relative_to(ROOT) else str(src), "bias": {}, "quant": {}}
    sys.path[:0] = [str(ROOT / "h1v2-isaac_amd"), str(ROOT / "oracle"), str(ROOT / "tests" / "helpers"),
                    str(ROOT / "tests")]
    from test_forced_harness import run_sole

    cpu_se = {}
    for f in sorted(src.glob("bias_*.json")):
        key = f.stem[len("bias_"):]
        d = json.loads(f.read_text())
        base = key[:-4] if key.endswith("_rsl") else key
        if base not in cpu_se:
            cpu_se[base] = run_sole(base, None).bias_fields()[2]
        out["bias"][key] = {n: float(f"{3 * abs(m) + 6 * max(s, c) + 1e-9:.3g}")
                            for n, m, s, c in zip(d["names"], d["mean"], d["se"], cpu_se[base])}
        out["quant"][key] = {c: [float(f"{2 * q['p50']:.2g}"), float(f"{2 * q['p99']:.2g}")] for c, q in d["quantiles"].items()}
    dst = ROOT / "tests" / "golden" / "sole_bias_gate.json"
    dst.write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print("wrote", dst, sorted(out["bias"]))


if __name__ == "__main__":
    main()
