"""CPU oracle for the avse_challenge hot path — TEST INFRASTRUCTURE ONLY.

This package is a plain PyTorch-CPU / numpy restatement of the reference's
algorithms (shangfuu/avse_challenge @ /root/reference, read-only).  It exists
to CHECK the MI355X HIP path, never to be the thing measured or shipped:

  * only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import it;
  * the product package ``avse_challenge_amd`` never imports it (a test
    enforces this), and fails loudly when its HIP library is missing.

Pinning: every restated function cites the reference file:line it follows.
The restatement is pinned against golden vectors produced by importing the
reference itself in the build container (``tests/golden/make_golden.py``;
the vectors are committed under ``tests/golden/``).  Where the arithmetic
lives in an un-vendored third-party package (mamba-ssm 1.1.3.post1,
causal-conv1d 1.1.3.post1, speechbrain 1.0.0, librosa 0.8.1) the restatement
follows that package's published algorithm and is marked "parity unpinned"
unless an in-tree reference definition pins it.
"""
