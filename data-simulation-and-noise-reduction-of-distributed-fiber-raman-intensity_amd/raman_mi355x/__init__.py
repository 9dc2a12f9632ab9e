"""raman_mi355x — MI355X-native (gfx950) batched inference engine for the Raman denoising networks
of 223qyc/Data-simulation-and-noise-reduction-of-distributed-fiber-Raman-intensity.

Drop-in surfaces (reference file:line):
  DenoiseCNN, RRCDNet, DSDN, ADSDN, PIDN, APIDN   */train.py model classes (models.py)
  generate_signals                                数据集产生.py:5-64 (simulator.py, on-device)
  evaluate, compute_*                             */evaulate.py:14-39 (evaluate.py, batched, on-device)
"""
from . import engine
from ._lib import EngineError, RangeError
from .dataset import load_dataset, save_dataset
from .distributed import all_reduce_sums, shard
from .evaluate import evaluate, write_metrics
from .models import ADSDN, APIDN, DSDN, MODELS, PIDN, DenoiseCNN, RRCDNet
from .simulator import generate, generate_signals

__all__ = ["engine", "DenoiseCNN", "RRCDNet", "DSDN", "ADSDN", "PIDN", "APIDN", "MODELS", "generate",
           "generate_signals", "evaluate", "write_metrics", "load_dataset", "save_dataset", "shard",
           "all_reduce_sums", "EngineError", "RangeError"]
