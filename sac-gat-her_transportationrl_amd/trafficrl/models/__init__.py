from .gat_encoder import GATConv, GATEncoder, global_max_pool, global_mean_pool  # noqa: F401
