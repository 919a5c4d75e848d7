// Key Vault with RBAC authorisation: JWT signing keys (security/jwt.py KeyVault signer) and OAuth
// client secrets (security/secrets.py azurekeyvault provider).  Readers get "Key Vault Secrets User".
param name string
param location string
param tags object
param readerPrincipalIds array
@description('Principals that write secrets at deployment time (the JWT key and OIDC app scripts)')
param writerPrincipalIds array = []
@allowed(['Enabled', 'Disabled'])
param publicNetworkAccess string = 'Enabled'

resource vault 'Microsoft.KeyVault/vaults@2023-07-01' = {
  name: name
  location: location
  tags: tags
  properties: {
    tenantId: subscription().tenantId
    sku: { family: 'A', name: 'standard' }
    enableRbacAuthorization: true
    enableSoftDelete: true
    softDeleteRetentionInDays: 30
    publicNetworkAccess: publicNetworkAccess
    networkAcls: { defaultAction: publicNetworkAccess == 'Enabled' ? 'Allow' : 'Deny', bypass: 'AzureServices' }
  }
}

var secretsUser = subscriptionResourceId('Microsoft.Authorization/roleDefinitions', '4633458b-17de-408a-b874-0445c86b69e6')

resource readers 'Microsoft.Authorization/roleAssignments@2022-04-01' = [for p in readerPrincipalIds: {
  name: guid(vault.id, p, secretsUser)
  scope: vault
  properties: { roleDefinitionId: secretsUser, principalId: p, principalType: 'ServicePrincipal' }
}]

// Key Vault Secrets Officer: the deployment scripts write the JWT key pair and the OIDC client secret
var secretsOfficer = subscriptionResourceId('Microsoft.Authorization/roleDefinitions', 'b86a8fe4-44ce-4948-aee5-eccb2c155cd7')

resource writers 'Microsoft.Authorization/roleAssignments@2022-04-01' = [for p in writerPrincipalIds: {
  name: guid(vault.id, p, secretsOfficer)
  scope: vault
  properties: { roleDefinitionId: secretsOfficer, principalId: p, principalType: 'ServicePrincipal' }
}]

output vaultUri string = vault.properties.vaultUri
output vaultName string = vault.name
output vaultId string = vault.id
