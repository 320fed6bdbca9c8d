"""psx.utils."""
