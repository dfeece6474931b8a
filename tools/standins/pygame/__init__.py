"""Stand-in: empty module (only the reference renderer uses pygame)."""
