"""Scoring runtime: compiled models, device plans, micro-batching engine, model cache."""
