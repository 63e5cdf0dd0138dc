#!/usr/bin/env python3
"""Render infrastructure/mi355x/cluster/scripts/cloud-init.tftpl without
Terraform (same substitution rules as ``templatefile`` for the subset the
template uses: ``${name}`` interpolation, ``$${`` escapes).

    python scripts/render_cloud_init.py --cluster-size 2 --repo-url URL --vm-username me \
        --ssh-public-key "ssh-ed25519 AAAA..." --out rendered/
"""
from __future__ import annotations

import argparse
import re
from pathlib import Path
from typing import Dict, List

TEMPLATE = Path(__file__).resolve().parent.parent / "infrastructure/mi355x/cluster/scripts/cloud-init.tftpl"

DEFAULTS = {
    "gpus_per_node": 8, "master_addr": "self", "master_port": 29500, "repo_dir": "distributed_training_amd",
    "entry": "src/multigpu_multi_node.py", "entry_args": "", "shared_mount": "/mnt/filesystem",
    "mount_command": "true",
}


def render(template: str, values: Dict[str, object]) -> str:
    def sub(m: re.Match) -> str:
        name = m.group(1)
        if name not in values:
            raise KeyError(f"template variable {name!r} not provided")
        return str(values[name])

    out = re.sub(r"(?<!\$)\$\{([A-Za-z_][A-Za-z0-9_]*)\}", sub, template)
    return out.replace("$${", "${")


def render_cluster(cluster_size: int, **kw) -> List[str]:
    if cluster_size <= 0:
        raise ValueError("Cluster size must be greater than 0")
    tpl = TEMPLATE.read_text()
    vals = {**DEFAULTS, **kw, "cluster_size": cluster_size}
    return [render(tpl, {**vals, "instance_index": i}) for i in range(cluster_size)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cluster-size", type=int, default=1)
    ap.add_argument("--vm-username", required=True)
    ap.add_argument("--ssh-public-key", required=True)
    ap.add_argument("--repo-url", required=True)
    ap.add_argument("--master-addr", default="self")
    ap.add_argument("--gpus-per-node", type=int, default=8)
    ap.add_argument("--entry-args", default="")
    ap.add_argument("--mount-command", default="true")
    ap.add_argument("--out", default="rendered")
    a = ap.parse_args()
    docs = render_cluster(a.cluster_size, vm_username=a.vm_username, ssh_public_key=a.ssh_public_key,
                          repo_url=a.repo_url, master_addr=a.master_addr, gpus_per_node=a.gpus_per_node,
                          entry_args=a.entry_args, mount_command=a.mount_command)
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    for i, d in enumerate(docs):
        (out / f"node-{i}.yaml").write_text(d)
        print(out / f"node-{i}.yaml")


if __name__ == "__main__":
    main()
