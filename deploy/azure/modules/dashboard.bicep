// Azure portal dashboard over the project's Application Insights: the pipeline's throughput and
// latency (the reference's metric names, pushed by the azure_monitor metrics driver) and the GPU
// side the reference does not have -- decode time to first token, HBM in use by the decoder and the
// vector index, KV cache bytes.  Each tile is an Application Insights metrics chart over customMetrics.
param base string
param location string
param tags object
param appInsightsId string

var charts = [
  { title: 'Summaries completed / min', metric: 'summarization_tokens_total', agg: 'Count' }
  { title: 'Summarization latency (s), p95 of the push interval', metric: 'summarization_latency_seconds', agg: 'Max' }
  { title: 'Chunks embedded', metric: 'embedding_chunks_processed_total', agg: 'Sum' }
  { title: 'Parsing duration (s)', metric: 'parsing_duration_seconds', agg: 'Avg' }
  { title: 'Decoder time to first token (s)', metric: 'summarization_gpu_ttft_seconds', agg: 'Avg' }
  { title: 'Decoder HBM in use (bytes)', metric: 'summarization_gpu_hbm_used_bytes', agg: 'Max' }
  { title: 'KV cache (bytes)', metric: 'summarization_gpu_kv_cache_bytes', agg: 'Max' }
  { title: 'Vector index on the GPU (bytes)', metric: 'copilot_vectorstore_device_bytes', agg: 'Max' }
  { title: 'Reporting API latency (s)', metric: 'reporting_http_request_duration_seconds', agg: 'Avg' }
]

resource dashboard 'Microsoft.Portal/dashboards@2020-09-01-preview' = {
  name: '${base}-pipeline'
  location: location
  tags: union(tags, { 'hidden-title': 'Copilot-for-Consensus on MI355X' })
  properties: {
    lenses: [
      {
        order: 0
        parts: [for (c, i) in charts: {
          position: { x: (i % 3) * 6, y: (i / 3) * 4, colSpan: 6, rowSpan: 4 }
          metadata: {
            type: 'Extension/HubsExtension/PartType/MonitorChartPart'
            inputs: [
              {
                name: 'options'
                value: {
                  chart: {
                    title: c.title
                    visualization: { chartType: 2 }
                    timespan: { relative: { duration: 86400000 } }
                    metrics: [
                      {
                        resourceMetadata: { id: appInsightsId }
                        name: 'customMetrics/${c.metric}'
                        aggregationType: c.agg == 'Sum' ? 1 : (c.agg == 'Count' ? 7 : (c.agg == 'Max' ? 3 : 4))
                        namespace: 'microsoft.insights/components/kusto'
                        metricVisualization: { displayName: c.metric }
                      }
                    ]
                  }
                }
              }
            ]
          }
        }]
      }
    ]
  }
}

output dashboardId string = dashboard.id
