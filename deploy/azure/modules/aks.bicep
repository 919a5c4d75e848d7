// AKS cluster: a CPU system pool for the gateway / ingestion / reporting / auth / UI pods and a
// GPU pool of AMD Instinct VMs for the encoder + HBM index + decoder pods (one process per GPU,
// torchrun over RCCL / xGMI inside a node).  The GPU pool is tainted so only the GPU workloads
// (deploy/k8s/copilot-mi355x.yaml, amd.com/gpu resource requests via the AMD device plugin) land
// there; KEDA scales the stage deployments on the Service Bus subscription backlogs (the
// reference's Container Apps scale rules); container insights go to the Log Analytics workspace.
param name string
param location string
param tags object
param systemVmSize string
param gpuVmSize string
param gpuNodeCount int
param logAnalyticsId string
param kubeletIdentityId string
@description('Subnet of both node pools (Azure CNI); empty = the cluster-managed network')
param subnetId string = ''

resource cluster 'Microsoft.ContainerService/managedClusters@2024-05-01' = {
  name: name
  location: location
  tags: tags
  identity: { type: 'UserAssigned', userAssignedIdentities: { '${kubeletIdentityId}': {} } }
  properties: {
    dnsPrefix: name
    enableRBAC: true
    oidcIssuerProfile: { enabled: true }
    securityProfile: { workloadIdentity: { enabled: true } }
    workloadAutoScalerProfile: { keda: { enabled: true } }
    addonProfiles: {
      omsagent: { enabled: true, config: { logAnalyticsWorkspaceResourceID: logAnalyticsId } }
    }
    // Azure CNI on the project vnet when a subnet is given: pods get vnet addresses and reach the
    // platform services through their private endpoints
    networkProfile: empty(subnetId) ? null : {
      networkPlugin: 'azure'
      networkPolicy: 'azure'
      serviceCidr: '10.1.0.0/16'
      dnsServiceIP: '10.1.0.10'
    }
    agentPoolProfiles: [
      {
        name: 'system'
        mode: 'System'
        vmSize: systemVmSize
        count: 2
        osType: 'Linux'
        osSKU: 'Ubuntu'
        vnetSubnetID: empty(subnetId) ? null : subnetId
      }
      {
        name: 'instinct'
        mode: 'User'
        vmSize: gpuVmSize
        count: gpuNodeCount
        osType: 'Linux'
        osSKU: 'Ubuntu'
        vnetSubnetID: empty(subnetId) ? null : subnetId
        nodeTaints: ['amd.com/gpu=present:NoSchedule']
        nodeLabels: { 'accelerator': 'amd-instinct' }
      }
    ]
  }
}

output clusterName string = cluster.name
output clusterId string = cluster.id
