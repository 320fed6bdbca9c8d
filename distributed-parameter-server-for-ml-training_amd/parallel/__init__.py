"""psx.parallel."""
