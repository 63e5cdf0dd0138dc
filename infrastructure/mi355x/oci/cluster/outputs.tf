# Same outputs as the reference cluster module (infrastructure/nebius/cluster/outputs.tf).
output "master_public_ip" {
  value = oci_core_instance.master.public_ip
}

output "master_internal_ip" {
  value = oci_core_instance.master.private_ip
}

output "worker_public_ips" {
  value = oci_core_instance.worker[*].public_ip
}

output "worker_internal_ips" {
  value = oci_core_instance.worker[*].private_ip
}

output "shared_filesystem" {
  value = "${oci_file_storage_mount_target.shared.ip_address}:/dta"
}
