"""Cross-cutting utilities: logging, metrics, profiling ranges, NUMA placement, config."""
