// Diagnostic settings: the platform services' resource logs and metrics go to the project's Log
// Analytics workspace next to the cluster's container insights and the services' Application
// Insights metrics, so one workspace answers "where did this thread stall" (Service Bus dead
// letters, Cosmos throttling, Key Vault denials, AKS control plane).
param workspaceId string
param cosmosName string
param serviceBusName string
param vaultName string
param storageName string
param aksName string

resource cosmos 'Microsoft.DocumentDB/databaseAccounts@2024-05-15' existing = { name: cosmosName }
resource bus 'Microsoft.ServiceBus/namespaces@2022-10-01-preview' existing = { name: serviceBusName }
resource vault 'Microsoft.KeyVault/vaults@2023-07-01' existing = { name: vaultName }
resource storage 'Microsoft.Storage/storageAccounts@2023-05-01' existing = { name: storageName }
resource blob 'Microsoft.Storage/storageAccounts/blobServices@2023-05-01' existing = { parent: storage, name: 'default' }
resource aks 'Microsoft.ContainerService/managedClusters@2024-05-01' existing = { name: aksName }

var allLogs = [{ categoryGroup: 'allLogs', enabled: true }]
var allMetrics = [{ category: 'AllMetrics', enabled: true }]

resource cosmosDiag 'Microsoft.Insights/diagnosticSettings@2021-05-01-preview' = {
  name: 'to-workspace'
  scope: cosmos
  properties: { workspaceId: workspaceId, logs: allLogs, metrics: allMetrics, logAnalyticsDestinationType: 'Dedicated' }
}

resource busDiag 'Microsoft.Insights/diagnosticSettings@2021-05-01-preview' = {
  name: 'to-workspace'
  scope: bus
  properties: { workspaceId: workspaceId, logs: allLogs, metrics: allMetrics }
}

resource vaultDiag 'Microsoft.Insights/diagnosticSettings@2021-05-01-preview' = {
  name: 'to-workspace'
  scope: vault
  properties: { workspaceId: workspaceId, logs: allLogs, metrics: allMetrics }
}

resource blobDiag 'Microsoft.Insights/diagnosticSettings@2021-05-01-preview' = {
  name: 'to-workspace'
  scope: blob
  properties: { workspaceId: workspaceId, logs: allLogs, metrics: [{ category: 'Transaction', enabled: true }] }
}

resource aksDiag 'Microsoft.Insights/diagnosticSettings@2021-05-01-preview' = {
  name: 'to-workspace'
  scope: aks
  properties: {
    workspaceId: workspaceId
    logs: [
      { category: 'kube-apiserver', enabled: true }
      { category: 'kube-audit-admin', enabled: true }
      { category: 'cluster-autoscaler', enabled: true }
    ]
    metrics: allMetrics
  }
}
