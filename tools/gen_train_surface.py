#!/usr/bin/env python3
"""Build-container only: the import / attribute surface the reference's training entry point touches, as DATA.

AST-parses the reference's scripts/rsl_rl/train.py and scripts/rsl_rl/cli_args.py (never imports or executes them)
and writes tests/golden/train_surface.json: every imported (module, name), every attribute path read or written on
the objects the script handles -- env_cfg, agent_cfg, args_cli, env / env.unwrapped, runner, app_launcher, the
classes it calls methods on -- the call keywords of the calls the drop-in must accept, and the decorator.  The
fixture holds names only (no source text); tests/test_train_surface.py resolves every entry against the shims, the
task / agent cfgs and the env class.

    python tools/gen_train_surface.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import ast
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "tests" / "golden" / "train_surface.json"
TRACKED = {"env_cfg", "agent_cfg", "args_cli", "env", "runner", "app_launcher", "simulation_app", "AppLauncher",
           "gym", "torch", "parser", "arg_group", "cli_args", "os", "sys"}


def attr_path(node):
    """'a.b.c' for an Attribute chain rooted at a Name, else None."""
    parts = []
    while isinstance(node, ast.Attribute):
        parts.append(node.attr)
        node = node.value
    if isinstance(node, ast.Name):
        return ".".join([node.id] + parts[::-1])
    return None


def scan(path: Path, rel: str) -> dict:
    tree = ast.parse(path.read_text(), filename=rel)
    imports, reads, writes, calls, decorators, dests = set(), set(), set(), {}, [], set()
    for node in ast.walk(tree):
        if isinstance(node, ast.ImportFrom) and node.module:
            for a in node.names:
                imports.add((node.module, a.name))
        elif isinstance(node, ast.Import):
            for a in node.names:
                imports.add((a.name, ""))
        elif isinstance(node, ast.Attribute):
            p = attr_path(node)
            if p and p.split(".")[0] in TRACKED:
                (writes if isinstance(node.ctx, ast.Store) else reads).add(p)
        elif isinstance(node, ast.Call):
            name = attr_path(node.func) if isinstance(node.func, ast.Attribute) else (
                node.func.id if isinstance(node.func, ast.Name) else None)
            if name and name.endswith("add_argument") and node.args and isinstance(node.args[0], ast.Constant):
                dests.add(str(node.args[0].value).lstrip("-").replace("-", "_"))
            if name:
                kws = sorted(k.arg for k in node.keywords if k.arg)
                c = calls.setdefault(name, {"nargs": set(), "keywords": set()})
                c["nargs"].add(len(node.args))
                c["keywords"].update(kws)
        elif isinstance(node, ast.FunctionDef):
            for d in node.decorator_list:
                if isinstance(d, ast.Call):
                    decorators.append({"function": node.name, "decorator": attr_path(d.func) or getattr(d.func, "id", None),
                                       "nargs": len(d.args), "args": [a.value if isinstance(a, ast.Constant)
                                                                      else attr_path(a) for a in d.args],
                                       "params": [a.arg for a in node.args.args]})
    # an attribute read that is only the prefix of a longer path adds nothing
    reads = {r for r in reads if not any(o != r and o.startswith(r + ".") for o in reads | writes)}
    return {"file": rel, "imports": sorted(map(list, imports)), "reads": sorted(reads), "writes": sorted(writes),
            "calls": {k: {"nargs": sorted(v["nargs"]), "keywords": sorted(v["keywords"])} for k, v in sorted(calls.items())},
            "decorators": decorators, "argparse_dests": sorted(dests)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    ref = Path(a.ref)
    out = {"source": "olivier-stasse/h1v2-Isaac scripts/rsl_rl/{train,cli_args}.py, AST names only (tools/gen_train_surface.py)",
           "scripts": [scan(ref / "scripts" / "rsl_rl" / f, f"scripts/rsl_rl/{f}") for f in ("train.py", "cli_args.py")]}
    OUT.write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print(f"wrote {OUT.relative_to(ROOT)}")


if __name__ == "__main__":
    main()
