output "rendered_user_data" {
  description = "cloud-init user-data per node (index 0 = master)"
  value       = local.user_data
}

output "rendered_files" {
  value = local_file.user_data[*].filename
}
