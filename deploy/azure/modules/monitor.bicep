// Log Analytics workspace (container insights of the cluster) + Application Insights (the
// azure_monitor metrics driver: the reference's metric names, observability/__init__.py).
param base string
param location string
param tags object

resource workspace 'Microsoft.OperationalInsights/workspaces@2023-09-01' = {
  name: '${base}-logs'
  location: location
  tags: tags
  properties: {
    sku: { name: 'PerGB2018' }
    retentionInDays: 30
  }
}

resource insights 'Microsoft.Insights/components@2020-02-02' = {
  name: '${base}-appi'
  location: location
  tags: tags
  kind: 'web'
  properties: {
    Application_Type: 'other'
    WorkspaceResourceId: workspace.id
  }
}

output workspaceId string = workspace.id
output appInsightsId string = insights.id
output appInsightsConnectionString string = insights.properties.ConnectionString
