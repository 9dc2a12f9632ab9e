"""Load the reference model classes / generator from /root/reference WITHOUT running the scripts.

Used ONLY by tests/golden/make_golden.py, in the build container, to produce committed fixtures.
Nothing under tests/ imports this at test time (the GPU box has no /root/reference).

Method: parse ``<model>/train.py`` with ``ast`` and exec only the ``ClassDef``
nodes (skipping ``RamanDataset``) into a namespace holding torch / nn / F / init.  A plain
``import train`` would run the whole training script at import time (train.py:32, :135, :158).
The generator is taken the same way: only the ``generate_signals`` FunctionDef of
数据集产生.py (:5-64) is exec'd; the module-level ``generate_all_datasets()`` (:88) is not.
"""
import ast
import os

REF = "/root/reference"

MODEL_DIRS = {
    "DenoiseCNN": "1DCNN",
    "RRCDNet": "RRCDNet",
    "DSDN": "DSDN",
    "ADSDN": "ADSDN",
    "PIDN": "PIDN",
    "APIDN": "APIDN",
}


def _exec_nodes(path, keep):
    import numpy as np
    import torch
    import torch.nn as nn
    import torch.nn.functional as F
    from torch.nn import init

    with open(path, encoding="utf-8") as fh:
        tree = ast.parse(fh.read(), filename=path)
    body = [n for n in tree.body if keep(n)]
    mod = ast.Module(body=body, type_ignores=[])
    ns = {"torch": torch, "nn": nn, "F": F, "init": init, "np": np}
    exec(compile(mod, path, "exec"), ns)
    return ns


def load_model_class(name):
    path = os.path.join(REF, MODEL_DIRS[name], "train.py")
    ns = _exec_nodes(path, lambda n: isinstance(n, ast.ClassDef) and n.name != "RamanDataset")
    return ns[name]


def load_generate_signals():
    path = os.path.join(REF, "数据集产生.py")
    ns = _exec_nodes(path, lambda n: isinstance(n, ast.FunctionDef) and n.name == "generate_signals")
    return ns["generate_signals"]
