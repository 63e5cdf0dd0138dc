# Single-MI355X development node -- the role of the reference's
# infrastructure/nebius/single_gpu (one GPU VM, no shared file system).  It
# boots with the same cloud-init as the cluster (../../cluster) set to one
# node and one rank, and runs the 1-GPU headline benchmark instead of the
# reference's commented-out training command.
locals {
  ssh_public_key = file(pathexpand(var.ssh_public_key_path))
}

resource "oci_core_vcn" "dev" {
  compartment_id = var.compartment_id
  cidr_blocks    = ["10.30.0.0/16"]
  display_name   = "dta-dev-vcn"
}

resource "oci_core_internet_gateway" "igw" {
  compartment_id = var.compartment_id
  vcn_id         = oci_core_vcn.dev.id
}

resource "oci_core_route_table" "public" {
  compartment_id = var.compartment_id
  vcn_id         = oci_core_vcn.dev.id
  route_rules {
    destination       = "0.0.0.0/0"
    network_entity_id = oci_core_internet_gateway.igw.id
  }
}

resource "oci_core_security_list" "dev" {
  compartment_id = var.compartment_id
  vcn_id         = oci_core_vcn.dev.id
  egress_security_rules {
    destination = "0.0.0.0/0"
    protocol    = "all"
  }
  ingress_security_rules {
    source   = var.ssh_source_cidr
    protocol = "6"
    tcp_options {
      min = 22
      max = 22
    }
  }
}

resource "oci_core_subnet" "dev" {
  compartment_id    = var.compartment_id
  vcn_id            = oci_core_vcn.dev.id
  cidr_block        = "10.30.1.0/24"
  route_table_id    = oci_core_route_table.public.id
  security_list_ids = [oci_core_security_list.dev.id]
}

module "boot" {
  source              = "../../cluster"
  vm_username         = var.vm_username
  ssh_public_key_path = var.ssh_public_key_path
  repo_url            = var.repo_url
  cluster_size        = 1
  gpus_per_node       = 1
  entry               = "bench.py"
  entry_args          = "--steps 2048 --warmup 256"
}

resource "oci_core_instance" "dev" {
  compartment_id      = var.compartment_id
  availability_domain = var.availability_domain
  shape               = var.gpu_shape
  display_name        = "dta-mi355x-dev"
  source_details {
    source_type             = "image"
    source_id               = var.image_id
    boot_volume_size_in_gbs = 256
  }
  create_vnic_details {
    subnet_id        = oci_core_subnet.dev.id
    assign_public_ip = true
  }
  metadata = {
    ssh_authorized_keys = local.ssh_public_key
    user_data           = base64encode(module.boot.rendered_user_data[0])
  }
}

output "public_ip" {
  value = oci_core_instance.dev.public_ip
}
