# Credentials come from the standard OCI provider environment / config file
# (OCI_CLI_* / ~/.oci/config), as the reference's Nebius provider reads
# NB_AUTHKEY_* (infrastructure/nebius/cluster/providers.tf).
provider "oci" {
  region = var.region
}
