"""dpgo_amd -- MI355X-native (gfx950, fp64 HIP) implementation of DPGO's Riemannian
block-coordinate-descent hot path (QuadraticProblem / LiftedSEManifold / QuadraticOptimizer as
driven by PGOAgent::updateX).  See DESIGN.md."""
__version__ = "0.1.0"
