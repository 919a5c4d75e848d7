// Storage account of the deployment scripts when they run inside the vnet (private networking):
// the script container mounts a file share from it, so it must admit the scripts subnet (service
// endpoint) and nothing else.  Deployment scripts authenticate to it with the account key.
param name string
param location string
param tags object
param subnetId string

resource account 'Microsoft.Storage/storageAccounts@2023-05-01' = {
  name: name
  location: location
  tags: tags
  kind: 'StorageV2'
  sku: { name: 'Standard_LRS' }
  properties: {
    minimumTlsVersion: 'TLS1_2'
    allowBlobPublicAccess: false
    allowSharedKeyAccess: true
    networkAcls: {
      defaultAction: 'Deny'
      bypass: 'AzureServices'
      virtualNetworkRules: [ { id: subnetId, action: 'Allow' } ]
    }
  }
}

output accountName string = account.name
