"""Kubernetes object subsets accepted in graph-component task options."""
