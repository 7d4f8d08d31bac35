"""Stand-in package for the absent deep-rl==0.2.9 (golden generation only)."""
