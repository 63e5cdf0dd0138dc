variable "vm_username" {
  type        = string
  description = "User created on every node"
}

variable "ssh_public_key_path" {
  type        = string
  description = "Public key authorised for that user"
  default     = "~/.ssh/id_ed25519.pub"
}

variable "cluster_size" {
  type        = number
  description = "Number of MI355X nodes (8 GPUs each)"
  default     = 1

  validation {
    condition     = var.cluster_size > 0
    error_message = "Cluster size must be greater than 0"
  }
}

variable "gpus_per_node" {
  type        = number
  description = "GPUs (ranks) per node"
  default     = 8
}

variable "master_addr" {
  type        = string
  description = "Private address of node 0 as the workers see it ('self' lets node 0 use its own address)"
  default     = "self"
}

variable "master_port" {
  type    = number
  default = 29500
}

variable "repo_url" {
  type        = string
  description = "Git URL of this repository"
}

variable "repo_dir" {
  type    = string
  default = "distributed_training_amd"
}

variable "entry" {
  type        = string
  description = "Training entrypoint launched by torchrun"
  default     = "src/multigpu_multi_node.py"
}

variable "entry_args" {
  type        = string
  description = "Arguments passed to the entrypoint (legacy CLI or key=value overrides)"
  default     = ""
}

variable "shared_mount" {
  type        = string
  description = "Mount point of the shared filesystem (checkpoints / outputs)"
  default     = "/mnt/filesystem"
}

variable "mount_command" {
  type        = string
  description = "Command that mounts the shared filesystem (provider specific: virtiofs, NFS, ...)"
  default     = "true"
}
