"""Test-only fault injection (SURVEY.md §5.3 plan: "kill rank r at step s").

``fault_injection: {rank: r, epoch: e, step: s, kind: exit|raise|hang, code: n}``
in the training config makes rank r fail at (epoch e, step s) so elastic
restart (``torchrun --max-restarts``) + snapshot resume can be exercised under
gloo on CPU.
"""
from __future__ import annotations

import logging
import os
import time
from typing import Dict

logger = logging.getLogger(__name__)


class InjectedFault(RuntimeError):
    pass


def inject_fault(spec: Dict) -> None:
    kind = spec.get("kind", "exit")
    marker = spec.get("once_marker")
    if marker:
        if os.path.exists(marker):
            return
        with open(marker, "w") as f:
            f.write("fired\n")
    logger.error(f"fault injection: {spec}")
    if kind == "raise":
        raise InjectedFault(f"injected fault {spec}")
    if kind == "hang":
        time.sleep(float(spec.get("seconds", 3600)))
        return
    os._exit(int(spec.get("code", 17)))
