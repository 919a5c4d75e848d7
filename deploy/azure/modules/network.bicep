// Project virtual network: one subnet for the AKS node pools (CPU system pool + AMD Instinct GPU
// pool, Azure CNI -- every pod gets a vnet address) and one for the private endpoints of the
// platform services (Cosmos DB, Key Vault, Storage, Service Bus Premium).  With private networking
// on, those services refuse public traffic and the pods reach them over these endpoints only.
param base string
param location string
param tags object

@description('Address space of the vnet')
param addressSpace string = '10.20.0.0/16'

@description('AKS nodes and pods (Azure CNI: size it for nodes x max pods)')
param aksSubnetPrefix string = '10.20.0.0/18'

@description('Private endpoints of the platform services')
param endpointSubnetPrefix string = '10.20.64.0/24'

@description('Deployment-script containers (JWT keys, OIDC app): they write Key Vault secrets, so with public access off they must run inside the vnet')
param scriptsSubnetPrefix string = '10.20.65.0/27'

var aksSubnetName = 'aks'
var endpointSubnetName = 'private-endpoints'
var scriptsSubnetName = 'deployment-scripts'

resource nsg 'Microsoft.Network/networkSecurityGroups@2024-01-01' = {
  name: '${base}-aks-nsg'
  location: location
  tags: tags
  properties: {
    securityRules: [
      {
        // the gateway is the only public entry (deploy/gateway: /reporting, /ingestion, /auth, /ui)
        name: 'allow-https-in'
        properties: {
          priority: 100
          direction: 'Inbound'
          access: 'Allow'
          protocol: 'Tcp'
          sourceAddressPrefix: 'Internet'
          sourcePortRange: '*'
          destinationAddressPrefix: '*'
          destinationPortRange: '443'
        }
      }
    ]
  }
}

resource vnet 'Microsoft.Network/virtualNetworks@2024-01-01' = {
  name: '${base}-vnet'
  location: location
  tags: tags
  properties: {
    addressSpace: { addressPrefixes: [addressSpace] }
    subnets: [
      {
        name: aksSubnetName
        properties: {
          addressPrefix: aksSubnetPrefix
          networkSecurityGroup: { id: nsg.id }
        }
      }
      {
        name: endpointSubnetName
        properties: {
          addressPrefix: endpointSubnetPrefix
          privateEndpointNetworkPolicies: 'Disabled'
        }
      }
      {
        // Azure Container Instances run the deployment scripts; the Storage service endpoint lets
        // them mount the scripts' file share from a storage account that admits this subnet only
        name: scriptsSubnetName
        properties: {
          addressPrefix: scriptsSubnetPrefix
          serviceEndpoints: [ { service: 'Microsoft.Storage' } ]
          delegations: [
            { name: 'aci', properties: { serviceName: 'Microsoft.ContainerInstance/containerGroups' } }
          ]
        }
      }
    ]
  }
}

output vnetId string = vnet.id
output aksSubnetId string = '${vnet.id}/subnets/${aksSubnetName}'
output endpointSubnetId string = '${vnet.id}/subnets/${endpointSubnetName}'
output scriptsSubnetId string = '${vnet.id}/subnets/${scriptsSubnetName}'
