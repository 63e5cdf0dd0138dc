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


def _hcl_blocks(text):
    """Top-level `resource "type" "name"` / `module "name"` / `variable "name"` headers of an HCL file."""
    return re.findall(r'^(resource|module|variable|output|data)\s+"([^"]+)"(?:\s+"([^"]+)")?\s*\{', text, re.M)


@pytest.mark.parametrize("mod", ["oci/cluster", "oci/single_gpu"])
def test_oci_modules_are_consistent(mod):
    """Provisioning modules (no terraform binary here): balanced braces, every var.X declared,
    every resource / module reference defined, boot module sources resolve."""
    d = ROOT / "infrastructure/mi355x" / mod
    text = {p.name: p.read_text() for p in d.glob("*.tf")}
    allt = "\n".join(text.values())
    for name, t in text.items():
        assert t.count("{") == t.count("}"), name
    blocks = _hcl_blocks(allt)
    declared_vars = {b[1] for b in blocks if b[0] == "variable"}
    for v in set(re.findall(r"\bvar\.([A-Za-z_]\w*)", allt)):
        assert v in declared_vars, v
    resources = {(b[1], b[2]) for b in blocks if b[0] == "resource"}
    for typ, name in set(re.findall(r"\b(oci_[a-z_]+)\.([a-z_0-9]+)\b", allt)):
        assert (typ, name) in resources, (typ, name)
    modules = {b[1]: None for b in blocks if b[0] == "module"}
    for m in set(re.findall(r"\bmodule\.([a-z_0-9]+)\b", allt)):
        assert m in modules, m
    for src in re.findall(r'source\s*=\s*"(\.[^"]+)"', allt):
        assert (d / src / "main.tf").exists(), src
    # the module passes exactly the boot module's variables
    boot_vars = {b[1] for b in _hcl_blocks((ROOT / "infrastructure/mi355x/cluster/variables.tf").read_text())}
    for body in re.findall(r'module\s+"[^"]+"\s*\{(.*?)\n\}', allt, re.S):
        for arg in re.findall(r"^\s*([a-z_]+)\s*=", body, re.M):
            assert arg == "source" or arg in boot_vars, arg


def test_oci_cluster_provisions_nodes_fabric_and_shared_fs():
    t = "\n".join(p.read_text() for p in (ROOT / "infrastructure/mi355x/oci/cluster").glob("*.tf"))
    kinds = {b[1] for b in _hcl_blocks(t) if b[0] == "resource"}
    for need in ("oci_core_instance", "oci_core_compute_cluster", "oci_file_storage_file_system",
                 "oci_file_storage_mount_target", "oci_file_storage_export", "oci_core_vcn", "oci_core_subnet"):
        assert need in kinds, need
    outs = {b[1] for b in _hcl_blocks(t) if b[0] == "output"}
    assert {"master_public_ip", "master_internal_ip", "worker_public_ips", "worker_internal_ips"} <= outs
    assert "count               = var.cluster_size - 1" in t and "depends_on = [oci_core_instance.master]" in t
