"""CPU oracle — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU, the reference algorithms of the hot path so that the HIP
engine can be checked against them:

* ``oracle.models``    — fp32 PyTorch-CPU functional forward of the six reference networks
  (1DCNN/train.py:71-82, RRCDNet/train.py:72-98, DSDN/train.py:72-126, ADSDN/train.py:72-167,
  PIDN/train.py:72-106, APIDN/train.py:72-159), driven straight from a ``state_dict``.
* ``oracle.weights``   — deterministic synthetic ``state_dict`` builder (numpy PCG64) used by the
  fixtures; BN running stats are randomised so that load-time folding is exercised.
* ``oracle.generator`` — numpy restatement of the engine's per-spectrum counter-based simulator
  (the distributional contract of 数据集产生.py:5-64), bit-exact on every integer draw.
* ``oracle.refgen``    — numpy restatement of the REFERENCE simulator's exact global-RNG draw order
  (数据集产生.py:5-64): regenerates the reference's data sets (config 1's ``data/test.npz``) bit for bit.
* ``oracle.metrics``   — numpy restatement of the evaluate.py metrics
  (*/evaulate.py:14-39 and skimage 0.18.3 ``structural_similarity`` with the reference's arguments).

Pinning: ``oracle.models`` and ``oracle.metrics`` are pinned against golden vectors produced from
the reference itself (tests/golden/make_golden.py loads the reference classes by AST extraction and
runs skimage 0.18.3 under /opt/conda/bin/python3.9), ``oracle.refgen`` against the inputs the
reference generator produced; see tests/test_cpu_host.py.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package, and only as the checker / CPU baseline — never as the product path.
"""
