"""CPU oracle for the CodeNeRF render/train hot path -- TEST INFRASTRUCTURE ONLY.

This package is the *checker*, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it.  The shipped path (``codenerf_amd``) never imports anything from
here and fails loudly when its HIP library is missing.

Contents
--------
``params``   seeded parameter init + canonical (reference state_dict) order.
``ref_cpu``  torch-CPU restatement of the reference algorithm
             (src/utils.py:10-47, src/model.py:4-53, src/trainer.py:61-85,
             torch.optim.AdamW as used at src/trainer.py:114-120).

Parity pinning
--------------
The restatement is pinned against golden vectors produced by importing the
reference's own ``src/model.py`` and ``src/utils.py`` in the build container
(``tools/gen_golden.py`` -> ``tests/golden/*.npz``); ``tests/test_oracle.py``
checks it against every fixture.  The reference ships no tests or fixtures of
its own, so those generated vectors are the only pin.
The fine (importance) sampling extension has no reference and is
"parity unpinned" (self-consistency only).
"""
