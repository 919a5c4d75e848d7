"""copilot_for_consensus_amd -- MI355X-native rebuild of Copilot-for-Consensus.

Control plane (Python): contracts, config, bus, storage, archive, parsing, chunking,
orchestration, reporting, services.  Data plane (HIP/CDNA4 + hipBLASLt + RCCL): models/, ops/,
runtime/, parallel/, vectorstore/ (see SURVEY.md §7 for the blueprint).
"""
__version__ = "0.1.0"
