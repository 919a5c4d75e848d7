// The auth service's RS256 signing key pair, generated once at deployment inside Azure and stored
// as Key Vault secrets `jwt-private-key` / `jwt-public-key` -- the names the local JWT signer's
// secret-sourced config reads (deploy/schemas/configs/adapters/drivers/jwt_signer/local.json:
// jwt_private_key / jwt_public_key; the azurekeyvault secret provider maps _ to -).  The script
// leaves an existing key pair alone (re-deployments keep issued tokens valid) unless `rotate`.
param location string
param tags object
param vaultName string
param identityId string

@minValue(2048)
param keyBits int = 3072

@description('Generate a new pair even when one exists (invalidates every issued token)')
param rotate bool = false

@description('Changes on every deployment so the (idempotent) script runs again')
param forceUpdateTag string = utcNow()

@description('Private networking: the script container joins this delegated subnet (the vault admits no public traffic)')
param subnetId string = ''

@description('Private networking: storage account for the script files, reachable from subnetId')
param storageAccountName string = ''

resource scriptStorage 'Microsoft.Storage/storageAccounts@2023-05-01' existing = if (!empty(storageAccountName)) {
  name: storageAccountName
}

resource keyScript 'Microsoft.Resources/deploymentScripts@2023-08-01' = {
  name: 'jwt-keys-${vaultName}'
  location: location
  tags: tags
  kind: 'AzureCLI'
  identity: { type: 'UserAssigned', userAssignedIdentities: { '${identityId}': {} } }
  properties: {
    azCliVersion: '2.61.0'
    forceUpdateTag: forceUpdateTag
    retentionInterval: 'PT1H'
    timeout: 'PT15M'
    cleanupPreference: 'OnSuccess'
    containerSettings: empty(subnetId) ? null : { subnetIds: [ { id: subnetId } ] }
    storageAccountSettings: empty(storageAccountName) ? null : {
      storageAccountName: storageAccountName
      storageAccountKey: scriptStorage.listKeys().keys[0].value
    }
    environmentVariables: [
      { name: 'VAULT', value: vaultName }
      { name: 'BITS', value: string(keyBits) }
      { name: 'ROTATE', value: rotate ? '1' : '0' }
    ]
    scriptContent: '''
      set -euo pipefail
      # RBAC role assignments on the vault can take a minute to reach the data plane; a vault
      # still unreachable after 5 minutes (role or network) fails the deployment here, instead of
      # reading as "no key" below
      ok=0
      for i in $(seq 1 20); do
        if az keyvault secret list --vault-name "$VAULT" -o none 2>/dev/null; then ok=1; break; fi
        sleep 15
      done
      if [ "$ok" != "1" ]; then echo "key vault $VAULT not reachable from the script" >&2; exit 1; fi
      if [ "$ROTATE" != "1" ] && az keyvault secret show --vault-name "$VAULT" -n jwt-private-key -o none 2>/dev/null; then
        echo "jwt key pair present: kept"
      else
        openssl genpkey -algorithm RSA -pkeyopt rsa_keygen_bits:"$BITS" -out key.pem
        openssl pkey -in key.pem -pubout -out pub.pem
        az keyvault secret set --vault-name "$VAULT" -n jwt-private-key -f key.pem -o none
        az keyvault secret set --vault-name "$VAULT" -n jwt-public-key -f pub.pem -o none
        shred -u key.pem
        echo "jwt key pair written"
      fi
      printf '{"privateKeySecret":"jwt-private-key","publicKeySecret":"jwt-public-key"}' > "$AZ_SCRIPTS_OUTPUT_PATH"
    '''
  }
}

output privateKeySecret string = keyScript.properties.outputs.privateKeySecret
output publicKeySecret string = keyScript.properties.outputs.publicKeySecret
