"""pongmi — the MI355X (gfx950) hot path of pingpong-selfplay-ai, behind the reference's own API.

  pongmi._lib      ctypes binding of libpongmi.so (include/pongmi.h); no CPU fallback
  pongmi.env       PongEnv2PBatch: n SoA fp64 arenas on the device (K1)
  pongmi.qnet      QNet parameter blocks + fused two-player acting (K2)
  pongmi.replay    prioritized replay sampling / priority update (K4)
  pongmi.selfplay  SelfPlayLearner: the batched train_iterative loop (K1+K2+K4+K3)
"""
from ._lib import PongmiError, load  # noqa: F401

__all__ = ["PongmiError", "load"]
