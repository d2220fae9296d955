"""CPU oracle for the MDX23C chunked-separation hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import it, and only as the checker / CPU timing baseline.
The product path (``sesa-audio-separation_amd/sesa``) never imports it and
fails loudly when its HIP library is missing.

Contents (each function cites the reference file:line it restates):

* ``oracle.weights``  -- name-keyed deterministic synthetic weights.
* ``oracle.mdx23c``   -- functional PyTorch-CPU fp32 restatement of
  ``models/mdx23c_tfc_tdf_v3.py`` (STFT, TFC_TDF blocks, TFC_TDF_net.forward).
* ``oracle.demix``    -- restatement of ``inference_pytorch.demix_pytorch_optimized``
  (chunker + windowed overlap-add), window/counter quirks included.
* ``oracle.ensemble`` -- restatement of ``ensemble.py`` blend methods.

Pinning: ``tests/golden/make_golden.py`` imports the *real* reference (in the
build container only, with stubbed third-party imports) and records golden
input/output vectors under ``tests/golden/*.npz``; ``tests/test_oracle.py``
checks this restatement against them.
"""
