"""CPU: the reference's own training entry point resolves on this build.

tests/golden/train_surface.json lists, as names only, what scripts/rsl_rl/train.py and scripts/rsl_rl/cli_args.py of
the reference import and touch (tools/gen_train_surface.py, an AST scan in the build container; the scripts are
never imported or run -- running them here was denied in round 1).  Every entry is resolved against
the import shims (h1v2-isaac_amd/shims), the task's env cfg and agent cfg as the registry returns them, the env
class and the runner:

* every imported (module, name) outside the standard library and the script's sibling cli_args;
* every attribute path read or written on env_cfg / agent_cfg (including what cli_args.update_rsl_rl_cfg writes),
  args_cli (the options train.py and cli_args define plus AppLauncher's), env / env.unwrapped, runner,
  app_launcher.app, gym;
* every call's positional count and keywords against the callee's signature;
* the @hydra_task_config(args_cli.task, "rsl_rl_cfg_entry_point") decorator on main(env_cfg, agent_cfg), driven with
  env.* / agent.* overrides in sys.argv as Hydra receives them after parse_known_args.
"""
import argparse
import importlib
import inspect
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SHIMS = ROOT / "h1v2-isaac_amd" / "shims"
SURFACE = json.loads((ROOT / "tests" / "golden" / "train_surface.json").read_text())
TRAIN, CLI = SURFACE["scripts"]
TASK = "Isaac-Velocity-Flat-H12_12dof-v0"
STDLIB = {"argparse", "os", "sys", "datetime", "typing", "__future__", "torch"}


@pytest.fixture(scope="module", autouse=True)
def shims():
    sys.path.insert(0, str(SHIMS))
    import biped_tasks.tasks  # noqa: F401  (registers the task ids, as train.py's import does)
    yield
    sys.path.remove(str(SHIMS))


def cfgs():
    from isaaclab_tasks.utils.parse_cfg import load_cfg_from_registry

    return load_cfg_from_registry(TASK, "env_cfg_entry_point"), load_cfg_from_registry(TASK, "rsl_rl_cfg_entry_point")


def resolve(obj, path):
    for k in path:
        obj = getattr(obj, k)
    return obj


def test_every_import_resolves():
    n = 0
    for s in (TRAIN, CLI):
        for mod, name in s["imports"]:
            if mod.split(".")[0] in STDLIB or mod == "cli_args":
                continue
            m = importlib.import_module(mod)
            if name:
                assert hasattr(m, name), f"{mod}.{name} ({s['file']})"
            n += 1
    assert n >= 15


def test_cfg_attribute_paths_resolve_and_are_writable():
    env_cfg, agent_cfg = cfgs()
    from h12env import H12FlatEnvCfg

    assert isinstance(env_cfg, H12FlatEnvCfg)
    roots = {"env_cfg": env_cfg, "agent_cfg": agent_cfg}
    seen = 0
    for s in (TRAIN, CLI):
        for kind in ("reads", "writes"):
            for p in s[kind]:
                root, *path = p.split(".")
                if root not in roots:
                    continue
                obj = resolve(roots[root], path[:-1])
                assert hasattr(obj, path[-1]), f"{p} ({s['file']} {kind})"
                if kind == "writes":
                    setattr(obj, path[-1], getattr(obj, path[-1]))
                seen += 1
    assert seen >= 20
    assert callable(agent_cfg.to_dict) and isinstance(agent_cfg.to_dict(), dict)


def test_args_cli_options_exist():
    from isaaclab.app import AppLauncher

    p = argparse.ArgumentParser()
    for d in TRAIN["argparse_dests"] + CLI["argparse_dests"]:
        p.add_argument(f"--{d}", default=None)
    AppLauncher.add_app_launcher_args(p)
    args, hydra = p.parse_known_args(["--task", TASK, "--num_envs", "64", "--headless", "env.scene.num_envs=32",
                                      "agent.max_iterations=3"])
    assert hydra == ["env.scene.num_envs=32", "agent.max_iterations=3"]
    for s in (TRAIN, CLI):
        for kind in ("reads", "writes"):
            for path in s[kind]:
                if path.startswith("args_cli."):
                    assert hasattr(args, path.split(".")[1]), f"{path} ({s['file']})"
    launcher = AppLauncher(args)
    assert callable(launcher.app.close)
    assert args.device is not None  # AppLauncher binds the device train.py reads into env_cfg.sim.device


def test_env_runner_and_call_signatures():
    import gymnasium as gym
    from h12env.env import H12VelocityEnv
    from isaaclab.envs import DirectMARLEnv
    from isaaclab.utils.dict import print_dict
    from isaaclab.utils.io import dump_pickle, dump_yaml
    from isaaclab_rl.rsl_rl import RslRlVecEnvWrapper
    from isaaclab_tasks.utils import get_checkpoint_path
    from isaaclab_tasks.utils.hydra import hydra_task_config
    from isaaclab.envs import multi_agent_to_single_agent
    from rsl_rl.runners import OnPolicyRunner

    assert inspect.isclass(DirectMARLEnv)
    # train.py reads env.unwrapped on the gym.make result and env.close on the RslRlVecEnvWrapper around it
    assert hasattr(H12VelocityEnv, "unwrapped") and hasattr(H12VelocityEnv, "close")
    assert hasattr(RslRlVecEnvWrapper, "close")
    for p in TRAIN["reads"]:
        if p.startswith("runner."):
            assert hasattr(OnPolicyRunner, p.split(".")[1]), p
        if p.startswith("gym."):
            assert resolve(gym, p.split(".")[1:]) is not None, p
    callees = {"OnPolicyRunner": OnPolicyRunner, "RslRlVecEnvWrapper": RslRlVecEnvWrapper, "gym.make": gym.make,
               "get_checkpoint_path": get_checkpoint_path, "dump_yaml": dump_yaml, "dump_pickle": dump_pickle,
               "print_dict": print_dict, "hydra_task_config": hydra_task_config,
               "multi_agent_to_single_agent": multi_agent_to_single_agent, "runner.learn": OnPolicyRunner.learn,
               "runner.load": OnPolicyRunner.load, "runner.add_git_repo_to_log": OnPolicyRunner.add_git_repo_to_log,
               "gym.wrappers.RecordVideo": gym.wrappers.RecordVideo}
    checked = 0
    for name, c in TRAIN["calls"].items():
        if name not in callees:
            continue
        f = callees[name]
        sig = inspect.signature(f)
        self_arg = 1 if name.startswith("runner.") else 0  # unbound method: the runner itself
        for nargs in c["nargs"]:
            sig.bind(*([None] * (nargs + self_arg)), **{k: None for k in c["keywords"]})
        checked += 1
    assert checked == len(callees)


def test_hydra_task_config_drives_main_with_overrides(monkeypatch):
    from isaaclab_tasks.utils.hydra import hydra_task_config

    dec = TRAIN["decorators"][0]
    assert dec["decorator"] == "hydra_task_config" and dec["args"] == ["args_cli.task", "rsl_rl_cfg_entry_point"]
    assert dec["params"] == ["env_cfg", "agent_cfg"]
    got = {}

    @hydra_task_config(TASK, dec["args"][1])
    def main(env_cfg, agent_cfg):
        got["env"], got["agent"] = env_cfg, agent_cfg

    # what train.py leaves in sys.argv for Hydra: the program name + the unknown (override) arguments
    monkeypatch.setattr(sys, "argv", ["train.py", "env.scene.num_envs=128", "env.sim.device=cuda:0",
                                      "agent.max_iterations=7", "agent.algorithm.learning_rate=0.0005",
                                      "agent.run_name=surface"])
    main()
    env_cfg, agent_cfg = got["env"], got["agent"]
    from h12env import H12FlatEnvCfg

    assert isinstance(env_cfg, H12FlatEnvCfg) and env_cfg.scene.num_envs == 128 and env_cfg.sim.device == "cuda:0"
    assert agent_cfg.max_iterations == 7 and agent_cfg.algorithm.learning_rate == 0.0005
    assert agent_cfg.run_name == "surface"
    # the rest of main()'s body, as train.py writes it
    env_cfg.seed = agent_cfg.seed
    d = agent_cfg.to_dict()
    assert d["max_iterations"] == 7 and d["algorithm"]["learning_rate"] == 0.0005
    monkeypatch.setattr(sys, "argv", ["train.py", "env.no_such_field=1"])
    with pytest.raises(AttributeError):
        main()
