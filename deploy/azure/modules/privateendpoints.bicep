// One private endpoint per platform service in the endpoint subnet, each registered in its
// private DNS zone (modules/privatedns.bicep).  `targets`: [{ name, resourceId, groupId, zoneId }]
// -- groupId 'Sql' (Cosmos NoSQL), 'vault', 'blob', 'namespace' (Service Bus Premium).
param base string
param location string
param tags object
param subnetId string
param targets array

resource endpoints 'Microsoft.Network/privateEndpoints@2024-01-01' = [for t in targets: {
  name: '${base}-${t.name}-pe'
  location: location
  tags: tags
  properties: {
    subnet: { id: subnetId }
    privateLinkServiceConnections: [
      {
        name: '${t.name}-link'
        properties: {
          privateLinkServiceId: t.resourceId
          groupIds: [t.groupId]
        }
      }
    ]
  }
}]

resource zoneGroups 'Microsoft.Network/privateEndpoints/privateDnsZoneGroups@2024-01-01' = [for (t, i) in targets: {
  parent: endpoints[i]
  name: 'default'
  properties: {
    privateDnsZoneConfigs: [{ name: t.name, properties: { privateDnsZoneId: t.zoneId } }]
  }
}]

output endpointIds array = [for (t, i) in targets: endpoints[i].id]
