#!/usr/bin/env python3
"""Gates of the sole-contact scenarios (tests/test_gpu_sensitivity.py::test_forced_sole_contact_scenarios).

Round 6: the signed-bias gate no longer inherits the kernel's own bias (round 5 used 3 x the kernel's measured |mean|).
Per scenario key and physics-state field

  bias[key][field] = 6 max(se, se_cpu) + 3 |m_f32| + 0.2 |m_hwt| + 1e-9

  se      the standard error of the kernel's signed mean (profiles/r6/bias_<key>.json, written by the test under
          H12_GATE_MEASURE=<dir> on the GPU): the resolution of the measurement, not its value
  se_cpu  that of tests/test_forced_harness.py's clean CPU stand-in (its rounding noise is calibrated to the kernel's
          floor, so the harness's clean run and the kernel pass by the same margin)
  m_f32   the signed mean of an independent fp32 evaluation of the same scenario: the oracle's own source in single
          precision (oracle/oracle_f32.c, tools/bias_attrib.py -> profiles/r6/bias_f32_oracle.json) -- what fp32
          arithmetic alone leaves in this statistic
  m_hwt   the same with the MI355X sin / cos error table (liboracle_f32hwt.so -> profiles/r6/bias_f32hwt_oracle.json):
          the bias the hardware's v_sin / v_cos put into an fp32 evaluation; the kernel removes its radial part to first
          order (fsincos), and a fifth of it covers what the first-order correction leaves (the kernel's measured
          remainder in stance is 15-17 % of the uncorrected bias)
  quant[key][crit] = (2 p50, 2 p99)  the kernel's absolute-error quantiles x2 (a noise floor, as in round 5)

The Rsl keys use the Flat scenario's fp32 references (the per-env friction spread does not change the fp32 evaluation).

    python tools/gen_sole_bias_gate.py [profiles/r6]
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main():
    src = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "profiles" / "r6"
    f32 = json.loads((ROOT / "profiles" / "r6" / "bias_f32_oracle.json").read_text())
    hwt = json.loads((ROOT / "profiles" / "r6" / "bias_f32hwt_oracle.json").read_text())
    out = {"source": str(src.relative_to(ROOT)) if src.is_relative_to(ROOT) else str(src),
           "formula": "6 max(se, se_cpu) + 3 |m_f32| + 0.2 |m_hwt| + 1e-9", "bias": {}, "quant": {}}
    sys.path[:0] = [str(ROOT / "h1v2-isaac_amd"), str(ROOT / "oracle"), str(ROOT / "tests" / "helpers"),
                    str(ROOT / "tests")]
    from test_forced_harness import run_sole

    cpu_se = {}
    for f in sorted(src.glob("bias_*.json")):
        key = f.stem[len("bias_"):]
        if key.startswith("f32"):
            continue
        d = json.loads(f.read_text())
        base = key[:-4] if key.endswith("_rsl") else key
        if base not in cpu_se:
            cpu_se[base] = run_sole(base, None).bias_fields()[2]
        idx = {n: i for i, n in enumerate(f32[base]["names"])}
        out["bias"][key] = {
            n: float(f"{6 * max(s, c) + 3 * abs(f32[base]['mean'][idx[n]]) + 0.2 * abs(hwt[base]['mean'][idx[n]]) + 1e-9:.3g}")
            for n, s, c in zip(d["names"], d["se"], cpu_se[base])}
        out["quant"][key] = {c: [float(f"{2 * q['p50']:.2g}"), float(f"{2 * q['p99']:.2g}")] for c, q in d["quantiles"].items()}
    dst = ROOT / "tests" / "golden" / "sole_bias_gate.json"
    dst.write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print("wrote", dst, sorted(out["bias"]))


if __name__ == "__main__":
    main()
