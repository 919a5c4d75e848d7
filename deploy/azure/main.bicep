// Copilot-for-Consensus on Azure, MI355X-native.
//
// The reference deploys its services as Container Apps (no GPU on that platform) next to
// Service Bus, Cosmos DB, Key Vault, Storage and Azure Monitor.  Here the GPU services run where
// AMD Instinct GPUs exist on Azure -- an AKS node pool of ND-series Instinct VMs (one process per
// GPU: services.main node under torchrun, or one pod per stage) -- and the platform services keep
// their roles and their names so the same drivers connect (cloud/azure.py):
//   * Service Bus: topic `copilot.events` + one subscription per consuming service, each filtered
//     on the routing keys it subscribes to (the RabbitMQ bindings of deploy/rabbitmq/definitions.json);
//   * Cosmos DB (NoSQL): database `copilot`, the six document collections, partition key /id;
//   * Storage: blob container `raw-archives` (archive store driver `azureblob`);
//   * Key Vault: JWT signing keys and OAuth secrets (secret provider `azurekeyvault`);
//   * Log Analytics + Application Insights (metrics driver `azure_monitor`);
//   * user-assigned identities with data-plane RBAC (no connection strings in pods);
//   * networking: a vnet (AKS subnet + private-endpoint subnet), private endpoints and private DNS
//     zones for Cosmos / Key Vault / Storage (and Service Bus on Premium), public access off;
//   * the auth service's RS256 key pair generated into Key Vault, an Entra ID app registration for
//     its Microsoft OIDC provider, diagnostic settings and a portal dashboard.
// Workloads: deploy/k8s/copilot-mi355x.yaml (KEDA scales the stages on subscription backlog).
targetScope = 'resourceGroup'

@description('Short prefix of every resource name')
@minLength(3)
@maxLength(12)
param projectName string = 'copilot'

@allowed(['dev', 'staging', 'prod'])
param environment string = 'dev'

param location string = resourceGroup().location

@description('VM size of the GPU node pool (AMD Instinct; the MI355X size when the region offers it)')
param gpuVmSize string = 'Standard_ND96isr_MI300X_v5'

@minValue(0)
param gpuNodeCount int = 1

@description('CPU node pool for the gateway, ingestion, reporting, auth and the UI')
param systemVmSize string = 'Standard_D8ds_v5'

@allowed(['Standard', 'Premium'])
param serviceBusSku string = 'Standard'

@minValue(400)
param cosmosMaxThroughput int = 4000

@description('Private endpoints + private DNS; the platform services refuse public traffic')
param enablePrivateNetworking bool = false

@description('Register an Entra ID app for the auth service (needs Graph Application.ReadWrite.OwnedBy)')
param enableEntraApp bool = false

@description('Public base URL of the gateway (OIDC redirect: <url>/auth/callback)')
param gatewayUrl string = ''

param tags object = {
  project: 'copilot-for-consensus'
  platform: 'mi355x'
}

var suffix = uniqueString(resourceGroup().id, projectName, environment)
var base = '${projectName}-${environment}'
var publicAccess = enablePrivateNetworking ? 'Disabled' : 'Enabled'
var sbPrivate = enablePrivateNetworking && serviceBusSku == 'Premium'
var aksSubnet = enablePrivateNetworking ? network.outputs.aksSubnetId : ''

module network 'modules/network.bicep' = if (enablePrivateNetworking) {
  name: 'network'
  params: { base: base, location: location, tags: tags }
}

module identities 'modules/identities.bicep' = {
  name: 'identities'
  params: { base: base, location: location, tags: tags }
}

module monitor 'modules/monitor.bicep' = {
  name: 'monitor'
  params: { base: base, location: location, tags: tags }
}

module keyVault 'modules/keyvault.bicep' = {
  name: 'keyvault'
  params: {
    name: take('${projectName}kv${suffix}', 24)
    location: location
    tags: tags
    readerPrincipalIds: [identities.outputs.servicesPrincipalId, identities.outputs.gpuPrincipalId]
    writerPrincipalIds: [identities.outputs.deployerPrincipalId]
    publicNetworkAccess: publicAccess
  }
}

module serviceBus 'modules/servicebus.bicep' = {
  name: 'servicebus'
  params: {
    name: '${base}-sb-${suffix}'
    location: location
    sku: serviceBusSku
    tags: tags
    principalIds: [identities.outputs.servicesPrincipalId, identities.outputs.gpuPrincipalId]
    publicNetworkAccess: sbPrivate ? 'Disabled' : 'Enabled'
  }
}

module cosmos 'modules/cosmos.bicep' = {
  name: 'cosmos'
  params: {
    name: '${base}-cosmos-${suffix}'
    location: location
    maxThroughput: cosmosMaxThroughput
    tags: tags
    principalIds: [identities.outputs.servicesPrincipalId, identities.outputs.gpuPrincipalId]
    publicNetworkAccess: publicAccess
  }
}

module storage 'modules/storage.bicep' = {
  name: 'storage'
  params: {
    name: take('${projectName}st${suffix}', 24)
    location: location
    tags: tags
    principalIds: [identities.outputs.servicesPrincipalId]
    publicNetworkAccess: publicAccess
  }
}

module aks 'modules/aks.bicep' = {
  name: 'aks'
  params: {
    name: '${base}-aks'
    location: location
    tags: tags
    systemVmSize: systemVmSize
    gpuVmSize: gpuVmSize
    gpuNodeCount: gpuNodeCount
    logAnalyticsId: monitor.outputs.workspaceId
    kubeletIdentityId: identities.outputs.gpuIdentityId
    subnetId: aksSubnet
  }
}

module privateDns 'modules/privatedns.bicep' = if (enablePrivateNetworking) {
  name: 'privatedns'
  params: { base: base, vnetId: network.outputs.vnetId, tags: tags, includeServiceBus: sbPrivate }
}

module privateEndpoints 'modules/privateendpoints.bicep' = if (enablePrivateNetworking) {
  name: 'privateendpoints'
  params: {
    base: base
    location: location
    tags: tags
    subnetId: network.outputs.endpointSubnetId
    targets: concat([
      { name: 'cosmos', resourceId: cosmos.outputs.accountId, groupId: 'Sql', zoneId: privateDns.outputs.zoneIds.cosmos }
      { name: 'vault', resourceId: keyVault.outputs.vaultId, groupId: 'vault', zoneId: privateDns.outputs.zoneIds.vault }
      { name: 'blob', resourceId: storage.outputs.accountId, groupId: 'blob', zoneId: privateDns.outputs.zoneIds.blob }
    ], sbPrivate ? [
      { name: 'servicebus', resourceId: serviceBus.outputs.namespaceId, groupId: 'namespace', zoneId: privateDns.outputs.zoneIds.servicebus }
    ] : [])
  }
}

// private networking: the deployment scripts write Key Vault secrets from inside the vnet (the vault
// refuses public traffic); their file share lives in a storage account that admits that subnet only
module scriptStorage 'modules/scriptstorage.bicep' = if (enablePrivateNetworking) {
  name: 'scriptstorage'
  params: {
    name: take('${projectName}ds${suffix}', 24)
    location: location
    tags: tags
    subnetId: network.outputs.scriptsSubnetId
  }
}

var scriptsSubnet = enablePrivateNetworking ? network.outputs.scriptsSubnetId : ''
var scriptsStorage = enablePrivateNetworking ? scriptStorage.outputs.accountName : ''

module jwtKeys 'modules/jwtkeys.bicep' = {
  name: 'jwtkeys'
  dependsOn: [privateEndpoints]
  params: {
    location: location
    tags: tags
    vaultName: keyVault.outputs.vaultName
    identityId: identities.outputs.deployerIdentityId
    subnetId: scriptsSubnet
    storageAccountName: scriptsStorage
  }
}

module oidcApp 'modules/oidc-app.bicep' = if (enableEntraApp) {
  name: 'oidc-app'
  params: {
    location: location
    tags: tags
    appName: '${base}-auth'
    redirectUris: ['${gatewayUrl}/auth/callback']
    vaultName: keyVault.outputs.vaultName
    identityId: identities.outputs.deployerIdentityId
    subnetId: scriptsSubnet
    storageAccountName: scriptsStorage
  }
  dependsOn: [privateEndpoints]
}

module diagnostics 'modules/diagnostics.bicep' = {
  name: 'diagnostics'
  params: {
    workspaceId: monitor.outputs.workspaceId
    cosmosName: '${base}-cosmos-${suffix}'
    serviceBusName: serviceBus.outputs.namespaceName
    vaultName: keyVault.outputs.vaultName
    storageName: storage.outputs.accountName
    aksName: aks.outputs.clusterName
  }
}

module dashboard 'modules/dashboard.bicep' = {
  name: 'dashboard'
  params: { base: base, location: location, tags: tags, appInsightsId: monitor.outputs.appInsightsId }
}

output serviceBusNamespace string = serviceBus.outputs.namespaceName
output serviceBusTopic string = serviceBus.outputs.topicName
output cosmosEndpoint string = cosmos.outputs.endpoint
output cosmosDatabase string = cosmos.outputs.databaseName
output storageAccount string = storage.outputs.accountName
output keyVaultUri string = keyVault.outputs.vaultUri
output appInsightsConnectionString string = monitor.outputs.appInsightsConnectionString
output aksName string = aks.outputs.clusterName
output jwtPrivateKeySecret string = jwtKeys.outputs.privateKeySecret
output oidcClientId string = enableEntraApp ? oidcApp.outputs.clientId : ''
output dashboardId string = dashboard.outputs.dashboardId
