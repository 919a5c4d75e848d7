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

@description('A new client secret is created only when the vault has none or it expires within this many days')
param renewDays int = 30

param forceUpdateTag string = utcNow()

@description('Private networking: the script container joins this delegated subnet (the vault admits no public traffic)')
param subnetId string = ''

@description('Private networking: storage account for the script files, reachable from subnetId')
param storageAccountName string = ''

resource scriptStorage 'Microsoft.Storage/storageAccounts@2023-05-01' existing = if (!empty(storageAccountName)) {
  name: storageAccountName
}

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
    containerSettings: empty(subnetId) ? null : { subnetIds: [ { id: subnetId } ] }
    storageAccountSettings: empty(storageAccountName) ? null : {
      storageAccountName: storageAccountName
      storageAccountKey: scriptStorage.listKeys().keys[0].value
    }
    environmentVariables: [
      { name: 'APP_NAME', value: appName }
      { name: 'RENEW_DAYS', value: string(renewDays) }
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
      client_id() { az keyvault secret set --vault-name "$VAULT" -n microsoft-oauth-client-id --value "$app" -o none; }
      # keep the current secret while it has more than RENEW_DAYS left (the vault secret carries its
      # expiry); otherwise add one, store it, then delete this app's older "copilot-auth" secrets,
      # so re-deployments never pile up valid client secrets
      end=$(az keyvault secret show --vault-name "$VAULT" -n microsoft-oauth-client-secret \
            --query attributes.expires -o tsv 2>/dev/null || true)
      if [ -n "$end" ] && [ "$(date -u -d "$end" +%s)" -gt "$(date -u -d "+${RENEW_DAYS} days" +%s)" ]; then
        client_id
        echo "client secret valid until $end: kept"
      else
        end=$(date -u -d "+${DAYS} days" +%Y-%m-%dT%H:%M:%SZ)
        secret=$(az ad app credential reset --id "$app" --append --display-name copilot-auth \
                 --end-date "$end" --query password -o tsv)
        client_id
        az keyvault secret set --vault-name "$VAULT" -n microsoft-oauth-client-secret --value "$secret" \
          --expires "$end" -o none
        newest=$(az ad app credential list --id "$app" \
                 --query "sort_by([?displayName=='copilot-auth'], &endDateTime)[-1].keyId" -o tsv)
        for k in $(az ad app credential list --id "$app" --query "[?displayName=='copilot-auth'].keyId" -o tsv); do
          if [ "$k" != "$newest" ]; then az ad app credential delete --id "$app" --key-id "$k"; fi
        done
        echo "client secret rotated, valid until $end"
      fi
      tenant=$(az account show --query tenantId -o tsv)
      printf '{"clientId":"%s","tenantId":"%s","secretExpires":"%s"}' "$app" "$tenant" "$end" > "$AZ_SCRIPTS_OUTPUT_PATH"
    '''
  }
}

output clientId string = appScript.properties.outputs.clientId
output tenantId string = appScript.properties.outputs.tenantId
output secretExpires string = appScript.properties.outputs.secretExpires
