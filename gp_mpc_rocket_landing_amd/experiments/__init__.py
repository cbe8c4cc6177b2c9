"""Monte-Carlo landing driver (reference src/experiments/monte_carlo.py)."""
