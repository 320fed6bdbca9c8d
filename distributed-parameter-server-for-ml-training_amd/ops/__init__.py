"""psx.ops."""
