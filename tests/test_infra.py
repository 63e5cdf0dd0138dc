"""Cluster bootstrap: cloud-init rendering and the
multi-node launcher, checked without a cloud or a GPU."""
import os
import re
import subprocess
import sys
from pathlib import Path

import pytest
import yaml

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scripts"))

from render_cloud_init import render, render_cluster  # noqa: E402


def _docs(n=3, **kw):
    return render_cluster(n, vm_username="trainer", ssh_public_key="ssh-ed25519 AAAAtest",
                          repo_url="https://example.invalid/dta.git", **kw)


def test_render_is_valid_cloud_config_per_node():
    docs = _docs(3, master_addr="10.0.0.5")
    assert len(docs) == 3
    for i, d in enumerate(docs):
        assert "${" not in d.replace("${NODE_RANK}", "")  # every template variable substituted
        cfg = yaml.safe_load(d)
        assert cfg["users"][0]["name"] == "trainer"
        script = cfg["write_files"][0]["content"]
        assert f"export NODE_RANK={i}" in script
        assert "export NNODES=3" in script
        assert "export MASTER_ADDR=10.0.0.5" in script
        assert "scripts/launch_multinode.sh" in script
        assert cfg["runcmd"][-1].endswith("setup_and_run.sh\"")


def test_rendered_setup_script_is_valid_bash(tmp_path):
    cfg = yaml.safe_load(_docs(2)[1])
    p = tmp_path / "setup.sh"
    p.write_text(cfg["write_files"][0]["content"])
    subprocess.run(["bash", "-n", str(p)], check=True)


def test_cluster_size_validation_and_missing_vars():
    with pytest.raises(ValueError):
        _docs(0)
    with pytest.raises(KeyError):
        render("${nope}", {})
    assert render("$${KEEP} ${a}", {"a": 1}) == "${KEEP} 1"


def _launch(env, *args):
    e = {**os.environ, "DRY_RUN": "1", "NPROC_PER_NODE": "8", **env}
    r = subprocess.run(["bash", str(ROOT / "scripts/launch_multinode.sh"), *args], env=e, capture_output=True,
                       text=True)
    return r


def test_launcher_master_and_worker_commands():
    r = _launch({"NNODES": "2", "NODE_RANK": "1", "MASTER_ADDR": "10.1.2.3"}, "10", "2", "--batch_size", "32")
    assert r.returncode == 0, r.stderr
    cmd = r.stdout.strip()
    for part in ("--nnodes=2", "--node_rank=1", "--master_addr=10.1.2.3", "--master_port=29500",
                 "--nproc_per_node=8", "src/multigpu_multi_node.py 10 2 --batch_size 32"):
        assert part in cmd
    assert "--max-restarts" not in cmd  # static rendezvous like the reference
    r = _launch({"NNODES": "1", "NODE_RANK": "0", "MAX_RESTARTS": "3", "MASTER_ADDR": "127.0.0.1"})
    assert "--max-restarts=3" in r.stdout


def test_launcher_worker_requires_master_addr():
    env = {k: v for k, v in os.environ.items() if k != "MASTER_ADDR"}
    r = subprocess.run(["bash", str(ROOT / "scripts/launch_multinode.sh")],
                       env={**env, "DRY_RUN": "1", "NNODES": "2", "NODE_RANK": "1", "NPROC_PER_NODE": "8"},
                       capture_output=True, text=True)
    assert r.returncode == 2 and "MASTER_ADDR is required" in r.stderr


def test_terraform_module_declares_template_variables():
    tpl = (ROOT / "infrastructure/mi355x/cluster/scripts/cloud-init.tftpl").read_text()
    names = set(re.findall(r"(?<!\$)\$\{([A-Za-z_]\w*)\}", tpl))
    main = (ROOT / "infrastructure/mi355x/cluster/main.tf").read_text()
    for n in names:
        assert re.search(rf"\b{n}\s*=", main), n
    variables = (ROOT / "infrastructure/mi355x/cluster/variables.tf").read_text()
    assert "var.cluster_size > 0" in variables
