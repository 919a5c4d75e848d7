#!/usr/bin/env bash
# Deploy the MI355X stack's Azure resources: ./deploy.sh <resource-group> <location> [dev|prod]
set -euo pipefail
rg="${1:?resource group}"; loc="${2:?location}"; env="${3:-dev}"
here="$(cd "$(dirname "$0")" && pwd)"
az group create --name "$rg" --location "$loc" --output none
az deployment group create --resource-group "$rg" --template-file "$here/main.bicep" \
  --parameters "@$here/parameters.$env.json" --parameters location="$loc" --output table
