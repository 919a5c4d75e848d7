// Microsoft Entra ID app registration for the auth service's "microsoft" OIDC provider
// (security/auth.py microsoft_provider; driver config oidc_providers/microsoft.json): a
// single-tenant web app with the gateway's /auth/callback redirect URIs, its client id and a client
// secret written to Key Vault as `microsoft-oauth-client-id` / `microsoft-oauth-client-secret`.
// Prerequisite (cannot be granted from a template): the deployment identity needs the Microsoft
// Graph application permission Application.ReadWrite.OwnedBy.
param location string
param tags object
param appName string
param redirectUris array
param vaultName string
param identityId string

@minValue(30)
@maxValue(730)
param secretDays int = 180

param forceUpdateTag string = utcNow()

resource appScript 'Microsoft.Resources/deploymentScripts@2023-08-01' = {
  name: 'oidc-app-${appName}'
  location: location
  tags: tags
  kind: 'AzureCLI'
  identity: { type: 'UserAssigned', userAssignedIdentities: { '${identityId}': {} } }
  properties: {
    azCliVersion: '2.61.0'
    forceUpdateTag: forceUpdateTag
    retentionInterval: 'PT1H'
    timeout: 'PT20M'
    cleanupPreference: 'OnSuccess'
    environmentVariables: [
      { name: 'APP_NAME', value: appName }
      { name: 'REDIRECTS', value: join(redirectUris, ' ') }
      { name: 'VAULT', value: vaultName }
      { name: 'DAYS', value: string(secretDays) }
    ]
    scriptContent: '''
      set -euo pipefail
      app=$(az ad app list --display-name "$APP_NAME" --query "[0].appId" -o tsv)
      if [ -z "$app" ]; then
        app=$(az ad app create --display-name "$APP_NAME" --sign-in-audience AzureADMyOrg \
              --web-redirect-uris $REDIRECTS --enable-id-token-issuance true --query appId -o tsv)
      else
        az ad app update --id "$app" --web-redirect-uris $REDIRECTS --enable-id-token-issuance true
      fi
      az ad sp show --id "$app" -o none 2>/dev/null || az ad sp create --id "$app" -o none
      end=$(date -u -d "+${DAYS} days" +%Y-%m-%dT%H:%M:%SZ)
      secret=$(az ad app credential reset --id "$app" --append --display-name copilot-auth \
               --end-date "$end" --query password -o tsv)
      az keyvault secret set --vault-name "$VAULT" -n microsoft-oauth-client-id --value "$app" -o none
      az keyvault secret set --vault-name "$VAULT" -n microsoft-oauth-client-secret --value "$secret" -o none
      tenant=$(az account show --query tenantId -o tsv)
      printf '{"clientId":"%s","tenantId":"%s","secretExpires":"%s"}' "$app" "$tenant" "$end" > "$AZ_SCRIPTS_OUTPUT_PATH"
    '''
  }
}

output clientId string = appScript.properties.outputs.clientId
output tenantId string = appScript.properties.outputs.tenantId
output secretExpires string = appScript.properties.outputs.secretExpires
