"""SiteWhere-AMD: an MI355X-native IoT application-enablement framework.

Capability parity with SiteWhere 2.0 (multitenant device registry, event
ingest/decoding, inbound processing, event persistence, enrichment, device
state/presence, rule processing, outbound connectors, command delivery,
assets, batch and scheduled operations, labels, streaming media, search,
REST + RPC APIs) with the event data plane running as fused CDNA4 kernels
on MI355X and sharded over RCCL/xGMI.  See docs/ARCHITECTURE.md.
"""
__version__ = "0.1.0"
