variable "region" {
  type        = string
  description = "OCI region with MI355X capacity"
}

variable "compartment_id" {
  type        = string
  description = "Compartment OCID for every resource"
}

variable "availability_domain" {
  type        = string
  description = "Availability domain of the GPU nodes (RDMA compute clusters are AD-local)"
}

variable "image_id" {
  type        = string
  description = "Ubuntu 22.04 image with ROCm 7.x and the AMD GPU driver (OCI GPU image or a custom one)"
}

variable "gpu_shape" {
  type        = string
  description = "Bare-metal 8x MI355X shape (8 GPUs fully connected by xGMI, RoCE NICs for the cluster fabric)"
  default     = "BM.GPU.MI355X.8"
}

variable "cluster_size" {
  type        = number
  description = "Number of 8-GPU nodes (node 0 is the torchrun master)"
  default     = 1

  validation {
    condition     = var.cluster_size > 0
    error_message = "Cluster size must be greater than 0"
  }
}

variable "vm_username" {
  type        = string
  description = "User created on every node by cloud-init"
}

variable "ssh_public_key_path" {
  type    = string
  default = "~/.ssh/id_ed25519.pub"
}

variable "repo_url" {
  type        = string
  description = "Git URL of this repository (cloned on every node)"
}

variable "entry" {
  type        = string
  description = "Entrypoint launched by torchrun on every node"
  default     = "src/multigpu_multi_node.py"
}

variable "entry_args" {
  type    = string
  default = ""
}

variable "boot_volume_gb" {
  type    = number
  default = 512
}

variable "shared_fs_mount" {
  type        = string
  description = "Mount point of the shared file system (checkpoints, Hydra outputs)"
  default     = "/mnt/filesystem"
}

variable "vcn_cidr" {
  type    = string
  default = "10.20.0.0/16"
}

variable "subnet_cidr" {
  type    = string
  default = "10.20.1.0/24"
}

variable "ssh_source_cidr" {
  type        = string
  description = "Where SSH to the nodes is allowed from"
  default     = "0.0.0.0/0"
}

variable "master_port" {
  type    = number
  default = 29500
}
