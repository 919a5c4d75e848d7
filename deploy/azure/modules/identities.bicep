// User-assigned identities: one for the CPU services, one for the GPU pods (kubelet + workload).
param base string
param location string
param tags object

resource services 'Microsoft.ManagedIdentity/userAssignedIdentities@2023-01-31' = {
  name: '${base}-services-id'
  location: location
  tags: tags
}

resource gpu 'Microsoft.ManagedIdentity/userAssignedIdentities@2023-01-31' = {
  name: '${base}-gpu-id'
  location: location
  tags: tags
}

// the deployment scripts' identity (JWT key generation, OIDC app registration)
resource deployer 'Microsoft.ManagedIdentity/userAssignedIdentities@2023-01-31' = {
  name: '${base}-deploy-id'
  location: location
  tags: tags
}

output deployerIdentityId string = deployer.id
output deployerPrincipalId string = deployer.properties.principalId
output servicesPrincipalId string = services.properties.principalId
output gpuPrincipalId string = gpu.properties.principalId
output gpuIdentityId string = gpu.id
