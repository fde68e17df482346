"""isaaclab.app.AppLauncher: there is no Omniverse app to launch; the launcher parses the same CLI
flags (headless, device, cameras, distributed) and binds the GPU of this rank."""
from __future__ import annotations

import argparse
import os
from types import SimpleNamespace


class AppLauncher:
    @staticmethod
    def add_app_launcher_args(parser: argparse.ArgumentParser) -> None:
        g = parser.add_argument_group("app_launcher", description="AppLauncher arguments (MI355X build: no simulator app)")
        g.add_argument("--headless", action="store_true", default=False)
        g.add_argument("--livestream", type=int, default=-1)
        g.add_argument("--enable_cameras", action="store_true", default=False)
        g.add_argument("--xr", action="store_true", default=False)
        g.add_argument("--device", type=str, default=None, help="cuda:<k> (default: cuda:LOCAL_RANK)")
        g.add_argument("--cpu", action="store_true", default=False)
        g.add_argument("--verbose", action="store_true", default=False)
        g.add_argument("--info", action="store_true", default=False)
        g.add_argument("--experience", type=str, default="")
        g.add_argument("--kit_args", type=str, default="")
        g.add_argument("--rendering_mode", type=str, default=None)
        if not any(a.dest == "distributed" for a in parser._actions):
            g.add_argument("--distributed", action="store_true", default=False)

    def __init__(self, launcher_args=None, **kwargs):
        if isinstance(launcher_args, argparse.Namespace):
            args = vars(launcher_args)
        else:
            args = dict(launcher_args or {})
        args.update(kwargs)
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.global_rank = int(os.environ.get("RANK", "0"))
        if args.get("device") is None and isinstance(launcher_args, argparse.Namespace):
            launcher_args.device = f"cuda:{self.local_rank}"
        if args.get("distributed"):
            import torch
            import torch.distributed as dist

            if not dist.is_initialized() and int(os.environ.get("WORLD_SIZE", "1")) > 1:
                torch.cuda.set_device(self.local_rank)
                dist.init_process_group("nccl", device_id=torch.device(f"cuda:{self.local_rank}"))
        self.app = SimpleNamespace(close=self._close, is_running=lambda: True, update=lambda: None)

    def _close(self):
        try:
            import torch.distributed as dist

            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:
            pass
