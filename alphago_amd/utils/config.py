"""Run configuration record (SURVEY.md §5 "Config / flag system").

The CLIs keep the reference's argparse flag names and defaults (Appendix B);
``RunConfig`` captures the parsed flags plus the execution environment
(world size, collective backend, device, kernel backend, library versions)
as one dataclass, serialised into native checkpoints and ``metadata.json``
so every artifact records how it was produced.
"""
from __future__ import annotations

import dataclasses
import os
import platform
from typing import Any, Dict, Optional


@dataclasses.dataclass
class RunConfig:
    command: str
    args: Dict[str, Any]
    world_size: int = 1
    dist_backend: str = "none"
    device: str = "cpu"
    kernel_backend: str = "auto"
    dtype: str = "bf16"
    torch_version: str = ""
    hip_version: Optional[str] = None
    host: str = ""

    @classmethod
    def capture(cls, command: str, args, env=None, kernel_backend: str = "auto", dtype: str = "bf16") -> "RunConfig":
        import torch

        a = vars(args) if hasattr(args, "__dict__") else dict(args)
        a = {k: (v if isinstance(v, (int, float, str, bool, type(None), list)) else str(v)) for k, v in a.items()}
        return cls(command=command, args=a,
                   world_size=getattr(env, "world_size", 1), dist_backend=getattr(env, "backend", "none"),
                   device=str(getattr(env, "device", "cpu")), kernel_backend=kernel_backend, dtype=dtype,
                   torch_version=str(torch.__version__),
                   hip_version=None if getattr(torch.version, "hip", None) is None else str(torch.version.hip),
                   host=os.environ.get("HOSTNAME", platform.node()))

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "RunConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})
