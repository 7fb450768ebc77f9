"""Shared utilities: env loading, logging, metrics and per-request tracing."""
