from .sac import Actor, Critic, DiscreteSAC, SACOutput, scatter_sum, segment_softmax  # noqa: F401
