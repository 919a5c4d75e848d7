// Private DNS zones of the platform services' private endpoints, each linked to the project vnet,
// so the drivers' ordinary host names (cosmos account, vault, blob account, Service Bus namespace)
// resolve to the endpoints' private addresses inside the cluster.
param base string
param vnetId string
param tags object

@description('Add the Service Bus zone (its private endpoint needs the Premium tier)')
param includeServiceBus bool = false

var core = environment().suffixes.storage
var zones = concat([
  { key: 'cosmos', zone: 'privatelink.documents.azure.com' }
  { key: 'vault', zone: 'privatelink.vaultcore.azure.net' }
  { key: 'blob', zone: 'privatelink.blob.${core}' }
], includeServiceBus ? [{ key: 'servicebus', zone: 'privatelink.servicebus.windows.net' }] : [])

resource dns 'Microsoft.Network/privateDnsZones@2020-06-01' = [for z in zones: {
  name: z.zone
  location: 'global'
  tags: tags
}]

resource links 'Microsoft.Network/privateDnsZones/virtualNetworkLinks@2020-06-01' = [for (z, i) in zones: {
  parent: dns[i]
  name: '${base}-${z.key}-link'
  location: 'global'
  tags: tags
  properties: {
    registrationEnabled: false
    virtualNetwork: { id: vnetId }
  }
}]

output zoneIds object = toObject(range(0, length(zones)), i => zones[i].key, i => dns[i].id)
