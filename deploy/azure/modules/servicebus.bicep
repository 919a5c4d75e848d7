// Service Bus: the event bus of the services (RabbitMQ's role; bus drivers in cloud/azure.py).
// One topic `copilot.events`; every message's subject is its routing key; each consuming service
// has one subscription whose SQL filter keeps exactly the routing keys it handles (the services'
// subscriptions(): ArchiveIngested -> parsing, JSONParsed -> chunking, ChunksPrepared -> embedding,
// EmbeddingsGenerated -> orchestrator, SummarizationRequested -> summarization, SummaryComplete ->
// reporting; SourceDeletionRequested fans out to the three cleaning stages).  Dead-lettering on
// filter errors and after maxDeliveryCount deliveries replaces the failed queues.
param name string
param location string
param sku string
param tags object
param principalIds array
@description('Disabled needs the Premium tier (private endpoint)')
@allowed(['Enabled', 'Disabled'])
param publicNetworkAccess string = 'Enabled'

var topicName = 'copilot.events'
var subscriptions = [
  { name: 'parsing', keys: ['archive.ingested', 'source.deletion.requested'] }
  { name: 'chunking', keys: ['json.parsed', 'source.deletion.requested'] }
  { name: 'embedding', keys: ['chunks.prepared', 'source.deletion.requested'] }
  { name: 'orchestrator', keys: ['embeddings.generated'] }
  { name: 'summarization', keys: ['summarization.requested'] }
  { name: 'reporting', keys: ['summary.complete'] }
]

resource ns 'Microsoft.ServiceBus/namespaces@2022-10-01-preview' = {
  name: name
  location: location
  tags: tags
  sku: { name: sku, tier: sku }
  properties: { disableLocalAuth: true, minimumTlsVersion: '1.2', publicNetworkAccess: publicNetworkAccess }
}

resource topic 'Microsoft.ServiceBus/namespaces/topics@2022-10-01-preview' = {
  parent: ns
  name: topicName
  properties: {
    defaultMessageTimeToLive: 'P14D'
    maxSizeInMegabytes: 5120
    requiresDuplicateDetection: true
    duplicateDetectionHistoryTimeWindow: 'PT10M'
  }
}

resource subs 'Microsoft.ServiceBus/namespaces/topics/subscriptions@2022-10-01-preview' = [for s in subscriptions: {
  parent: topic
  name: s.name
  properties: {
    lockDuration: 'PT5M'
    maxDeliveryCount: 8
    deadLetteringOnMessageExpiration: true
    deadLetteringOnFilterEvaluationExceptions: true
  }
}]

resource rules 'Microsoft.ServiceBus/namespaces/topics/subscriptions/rules@2022-10-01-preview' = [for (s, i) in subscriptions: {
  parent: subs[i]
  name: 'routing-keys'
  properties: {
    filterType: 'SqlFilter'
    sqlFilter: { sqlExpression: 'sys.Label IN (\'${join(s.keys, '\', \'')}\')' }
  }
}]

// Azure Service Bus Data Owner (send + receive) for the service identities
var dataOwner = subscriptionResourceId('Microsoft.Authorization/roleDefinitions', '090c5cfd-751d-490a-894a-3ce6f1109419')

resource access 'Microsoft.Authorization/roleAssignments@2022-04-01' = [for p in principalIds: {
  name: guid(ns.id, p, dataOwner)
  scope: ns
  properties: { roleDefinitionId: dataOwner, principalId: p, principalType: 'ServicePrincipal' }
}]

output namespaceName string = ns.name
output topicName string = topic.name
output namespaceId string = ns.id
