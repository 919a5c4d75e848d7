// Storage account: the archive store (archive/__init__.py azureblob driver, container raw-archives)
// and the HBM vector index snapshots (vectorstore save / load: safetensors + row-table .npy).
param name string
param location string
param tags object
param principalIds array
@allowed(['Enabled', 'Disabled'])
param publicNetworkAccess string = 'Enabled'

resource account 'Microsoft.Storage/storageAccounts@2023-05-01' = {
  name: name
  location: location
  tags: tags
  sku: { name: 'Standard_ZRS' }
  kind: 'StorageV2'
  properties: {
    allowBlobPublicAccess: false
    allowSharedKeyAccess: false
    minimumTlsVersion: 'TLS1_2'
    supportsHttpsTrafficOnly: true
    publicNetworkAccess: publicNetworkAccess
  }
}

resource blobs 'Microsoft.Storage/storageAccounts/blobServices@2023-05-01' = {
  parent: account
  name: 'default'
}

resource archives 'Microsoft.Storage/storageAccounts/blobServices/containers@2023-05-01' = {
  parent: blobs
  name: 'raw-archives'
}

resource indexSnapshots 'Microsoft.Storage/storageAccounts/blobServices/containers@2023-05-01' = {
  parent: blobs
  name: 'vector-index'
}

// Storage Blob Data Contributor
var blobContributor = subscriptionResourceId('Microsoft.Authorization/roleDefinitions', 'ba92f5b4-2d11-453d-a403-e96b0029c9fe')

resource access 'Microsoft.Authorization/roleAssignments@2022-04-01' = [for p in principalIds: {
  name: guid(account.id, p, blobContributor)
  scope: account
  properties: { roleDefinitionId: blobContributor, principalId: p, principalType: 'ServicePrincipal' }
}]

output accountName string = account.name
output accountId string = account.id
