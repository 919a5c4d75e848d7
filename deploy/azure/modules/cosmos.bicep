// Cosmos DB (NoSQL API): the document store (storage/document_store.py cosmos driver).  Database
// `copilot`, one container per document collection (contracts/documents.py COLLECTIONS), partition
// key /id (every access is by _id or a filtered scan, as the reference's store), autoscale
// throughput shared at the database level; data-plane RBAC (no keys in the pods).
param name string
param location string
param maxThroughput int
param tags object
param principalIds array
@allowed(['Enabled', 'Disabled'])
param publicNetworkAccess string = 'Enabled'

var databaseName = 'copilot'
var collections = ['archives', 'messages', 'threads', 'chunks', 'summaries', 'sources']

resource account 'Microsoft.DocumentDB/databaseAccounts@2024-05-15' = {
  name: name
  location: location
  tags: tags
  kind: 'GlobalDocumentDB'
  properties: {
    databaseAccountOfferType: 'Standard'
    consistencyPolicy: { defaultConsistencyLevel: 'Session' }
    locations: [{ locationName: location, failoverPriority: 0 }]
    disableLocalAuth: true
    publicNetworkAccess: publicNetworkAccess
  }
}

resource db 'Microsoft.DocumentDB/databaseAccounts/sqlDatabases@2024-05-15' = {
  parent: account
  name: databaseName
  properties: {
    resource: { id: databaseName }
    options: { autoscaleSettings: { maxThroughput: maxThroughput } }
  }
}

resource containers 'Microsoft.DocumentDB/databaseAccounts/sqlDatabases/containers@2024-05-15' = [for c in collections: {
  parent: db
  name: c
  properties: {
    resource: {
      id: c
      partitionKey: { paths: ['/id'], kind: 'Hash' }
      indexingPolicy: { indexingMode: 'consistent', includedPaths: [{ path: '/*' }] }
    }
  }
}]

// Cosmos DB Built-in Data Contributor
resource rbac 'Microsoft.DocumentDB/databaseAccounts/sqlRoleAssignments@2024-05-15' = [for p in principalIds: {
  parent: account
  name: guid(account.id, p, 'data-contributor')
  properties: {
    roleDefinitionId: '${account.id}/sqlRoleDefinitions/00000000-0000-0000-0000-000000000002'
    principalId: p
    scope: account.id
  }
}]

output endpoint string = account.properties.documentEndpoint
output databaseName string = db.name
output accountId string = account.id
