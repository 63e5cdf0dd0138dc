variable "region" {
  type = string
}

variable "compartment_id" {
  type = string
}

variable "availability_domain" {
  type = string
}

variable "image_id" {
  type        = string
  description = "Ubuntu 22.04 image with ROCm 7.x"
}

variable "gpu_shape" {
  type        = string
  description = "MI355X shape for the dev node (the smallest MI355X shape the region offers)"
  default     = "BM.GPU.MI355X.8"
}

variable "vm_username" {
  type = string
}

variable "ssh_public_key_path" {
  type    = string
  default = "~/.ssh/id_ed25519.pub"
}

variable "repo_url" {
  type = string
}

variable "ssh_source_cidr" {
  type    = string
  default = "0.0.0.0/0"
}
