"""Utilities outside the hot path: model store (local dir / GCS) and offline evaluation."""
