"""MI355X-native FiBiNET CTR training path (drop-in for YOUNESELBOUKNIFY/Ctr_recommendation).

Public modules:
  model_fibinet  -- build_model / MM_FiBiNET (drop-in for src/model_fibinet.py)
  trainer        -- FiBiNETTrainer: fused native train step (clip + Adam + OneCycleLR on device,
                    row-sharded multi-GPU)
  utils          -- set_seed / compute_auc / compute_logloss (src/utils.py)
  data           -- MicroLens-shaped synthetic batches
The compute lives in libfibinet_hip.so (csrc/, C ABI in include/fibinet.h).
"""
__version__ = "0.1.0"
