terraform {
  required_version = ">= 1.3"
  required_providers {
    oci = {
      source  = "oracle/oci"
      version = ">= 5.30"
    }
    local = {
      source  = "hashicorp/local"
      version = ">= 2.4"
    }
  }
}
