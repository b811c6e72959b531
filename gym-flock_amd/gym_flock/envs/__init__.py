"""Env packages mirroring the reference's gym_flock/envs layout."""
