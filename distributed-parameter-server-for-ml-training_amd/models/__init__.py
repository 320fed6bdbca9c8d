"""psx.models."""
