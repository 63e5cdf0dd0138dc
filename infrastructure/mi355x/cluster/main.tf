# Provider-agnostic MI355X cluster bootstrap.
#
# The reference provisions Nebius H100 VMs directly
# (infrastructure/nebius/cluster/main.tf).  MI355X capacity comes from several
# clouds with different instance resources, so this module renders the
# per-node cloud-init user-data (node 0 = master, 1..N-1 = workers) and
# leaves instance creation to a thin provider-specific wrapper that passes
# `rendered_user_data[i]` as the user-data of node i, e.g.
#
#   module "boot" { source = "./infrastructure/mi355x/cluster" ... }
#   resource "<provider>_instance" "node" {
#     count     = var.cluster_size
#     user_data = module.boot.rendered_user_data[count.index]
#     ...       # 8x MI355X shape, ROCm image, shared filesystem attachment
#   }
locals {
  ssh_public_key = file(pathexpand(var.ssh_public_key_path))
  user_data = [
    for i in range(var.cluster_size) : templatefile("${path.module}/scripts/cloud-init.tftpl", {
      vm_username    = var.vm_username
      ssh_public_key = local.ssh_public_key
      repo_url       = var.repo_url
      repo_dir       = var.repo_dir
      cluster_size   = var.cluster_size
      instance_index = i
      master_addr    = var.master_addr
      master_port    = var.master_port
      gpus_per_node  = var.gpus_per_node
      entry          = var.entry
      entry_args     = var.entry_args
      shared_mount   = var.shared_mount
      mount_command  = var.mount_command
    })
  ]
}

resource "local_file" "user_data" {
  count    = var.cluster_size
  filename = "${path.module}/rendered/node-${count.index}.yaml"
  content  = local.user_data[count.index]
}
