# Multi-node MI355X cluster on OCI bare metal -- the role of the reference's
# infrastructure/nebius/cluster/main.tf (master + workers on a GPU cluster
# fabric, shared file system for checkpoints, per-node cloud-init that starts
# torchrun), re-designed for 8x MI355X nodes:
#
#   * nodes: BM.GPU.MI355X.8 (8 GPUs per node, xGMI inside the node -- the
#     intra-node collectives never leave it), one torchrun with 8 ranks each;
#   * fabric: an RDMA compute cluster (RoCE between nodes; RCCL's net plugin
#     uses it for the inter-node steps of its collectives), the counterpart of
#     the reference's `nebius_compute_v1_gpu_cluster` on IB fabric-3;
#   * shared storage: an FSS file system + mount target exported to the
#     subnet and mounted over NFS at var.shared_fs_mount on every node (the
#     reference attaches a virtiofs NETWORK_SSD filesystem);
#   * boot: the provider-agnostic cloud-init of ../../cluster (user, clone,
#     native build, master wait on the rendezvous port, torchrun), one
#     document per node, node 0 = master, workers get node 0's private IP.
locals {
  ssh_public_key = file(pathexpand(var.ssh_public_key_path))
  nfs_mount      = "mkdir -p ${var.shared_fs_mount} && mount -t nfs -o vers=3,nconnect=16 ${oci_file_storage_mount_target.shared.ip_address}:/dta ${var.shared_fs_mount}"
}

# ------------------------------------------------------------------ network
resource "oci_core_vcn" "cluster" {
  compartment_id = var.compartment_id
  cidr_blocks    = [var.vcn_cidr]
  display_name   = "dta-mi355x-vcn"
  dns_label      = "dtami355x"
}

resource "oci_core_internet_gateway" "igw" {
  compartment_id = var.compartment_id
  vcn_id         = oci_core_vcn.cluster.id
  display_name   = "dta-igw"
}

resource "oci_core_route_table" "public" {
  compartment_id = var.compartment_id
  vcn_id         = oci_core_vcn.cluster.id
  route_rules {
    destination       = "0.0.0.0/0"
    network_entity_id = oci_core_internet_gateway.igw.id
  }
}

resource "oci_core_security_list" "cluster" {
  compartment_id = var.compartment_id
  vcn_id         = oci_core_vcn.cluster.id
  display_name   = "dta-cluster"

  egress_security_rules {
    destination = "0.0.0.0/0"
    protocol    = "all"
  }
  # everything between the nodes: torchrun rendezvous (master_port), RCCL
  # bootstrap / socket transport, NFS to the mount target
  ingress_security_rules {
    source   = var.subnet_cidr
    protocol = "all"
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

resource "oci_core_subnet" "cluster" {
  compartment_id    = var.compartment_id
  vcn_id            = oci_core_vcn.cluster.id
  cidr_block        = var.subnet_cidr
  display_name      = "dta-cluster-subnet"
  dns_label         = "nodes"
  route_table_id    = oci_core_route_table.public.id
  security_list_ids = [oci_core_security_list.cluster.id]
}

# ------------------------------------------------------------------ fabric
resource "oci_core_compute_cluster" "rdma" {
  compartment_id      = var.compartment_id
  availability_domain = var.availability_domain
  display_name        = "dta-mi355x-rdma"
}

# ------------------------------------------------------------------ shared file system
resource "oci_file_storage_file_system" "shared" {
  compartment_id      = var.compartment_id
  availability_domain = var.availability_domain
  display_name        = "dta-shared"
}

resource "oci_file_storage_mount_target" "shared" {
  compartment_id      = var.compartment_id
  availability_domain = var.availability_domain
  subnet_id           = oci_core_subnet.cluster.id
  display_name        = "dta-shared-mt"
}

resource "oci_file_storage_export" "shared" {
  export_set_id  = oci_file_storage_mount_target.shared.export_set_id
  file_system_id = oci_file_storage_file_system.shared.id
  path           = "/dta"
  export_options {
    source          = var.subnet_cidr
    access          = "READ_WRITE"
    identity_squash = "NONE"
  }
}

# ------------------------------------------------------------------ boot documents
module "boot_master" {
  source              = "../../cluster"
  vm_username         = var.vm_username
  ssh_public_key_path = var.ssh_public_key_path
  repo_url            = var.repo_url
  cluster_size        = var.cluster_size
  gpus_per_node       = 8
  master_addr         = "self"
  master_port         = var.master_port
  entry               = var.entry
  entry_args          = var.entry_args
  shared_mount        = var.shared_fs_mount
  mount_command       = local.nfs_mount
}

module "boot_workers" {
  source              = "../../cluster"
  vm_username         = var.vm_username
  ssh_public_key_path = var.ssh_public_key_path
  repo_url            = var.repo_url
  cluster_size        = var.cluster_size
  gpus_per_node       = 8
  master_addr         = oci_core_instance.master.private_ip
  master_port         = var.master_port
  entry               = var.entry
  entry_args          = var.entry_args
  shared_mount        = var.shared_fs_mount
  mount_command       = local.nfs_mount
}

# ------------------------------------------------------------------ nodes
resource "oci_core_instance" "master" {
  compartment_id      = var.compartment_id
  availability_domain = var.availability_domain
  compute_cluster_id  = oci_core_compute_cluster.rdma.id
  shape               = var.gpu_shape
  display_name        = "dta-node-0"

  source_details {
    source_type             = "image"
    source_id               = var.image_id
    boot_volume_size_in_gbs = var.boot_volume_gb
  }
  create_vnic_details {
    subnet_id        = oci_core_subnet.cluster.id
    assign_public_ip = true
    hostname_label   = "node0"
  }
  metadata = {
    ssh_authorized_keys = local.ssh_public_key
    user_data           = base64encode(module.boot_master.rendered_user_data[0])
  }
  depends_on = [oci_file_storage_export.shared]
}

resource "oci_core_instance" "worker" {
  count               = var.cluster_size - 1
  compartment_id      = var.compartment_id
  availability_domain = var.availability_domain
  compute_cluster_id  = oci_core_compute_cluster.rdma.id
  shape               = var.gpu_shape
  display_name        = "dta-node-${count.index + 1}"

  source_details {
    source_type             = "image"
    source_id               = var.image_id
    boot_volume_size_in_gbs = var.boot_volume_gb
  }
  create_vnic_details {
    subnet_id        = oci_core_subnet.cluster.id
    assign_public_ip = true
    hostname_label   = "node${count.index + 1}"
  }
  metadata = {
    ssh_authorized_keys = local.ssh_public_key
    user_data           = base64encode(module.boot_workers.rendered_user_data[count.index + 1])
  }
  # workers start after the master exists (they wait for its rendezvous port in cloud-init)
  depends_on = [oci_core_instance.master]
}
