"""Cross-cutting utilities: tracing, stats, logging, config, system info."""
