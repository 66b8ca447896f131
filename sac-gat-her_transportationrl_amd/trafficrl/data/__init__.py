from .tntp_parser import EdgeData, GraphData, load_graph_data, parse_net_tntp, parse_trips_tntp, sioux_falls  # noqa: F401
from .synthetic import anaheim_synthetic, synthetic_network, write_tntp  # noqa: F401
