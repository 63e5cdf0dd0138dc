# Single-MI355X development VM (role of the reference's
# infrastructure/nebius/single_gpu): one node, one rank, running the 1-GPU
# smoke + benchmark instead of a commented-out training command.
module "node" {
  source              = "../cluster"
  vm_username         = var.vm_username
  ssh_public_key_path = var.ssh_public_key_path
  repo_url            = var.repo_url
  cluster_size        = 1
  gpus_per_node       = 1
  entry               = "bench.py"
  entry_args          = "--steps 2048 --warmup 256"
}

output "rendered_user_data" {
  value = module.node.rendered_user_data[0]
}
