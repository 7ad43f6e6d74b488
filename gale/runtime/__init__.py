"""gale runtime: model replicas (plan executor + hipGraphs) and the streaming engine."""
