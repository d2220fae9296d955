"""Restatement of the third-party ``demucs`` package pieces HTDemucs uses.  TEST INFRASTRUCTURE ONLY
(oracle/): never imported by the product path.

``models/demucs4ht.py:10-25`` imports ``demucs.{demucs, hdemucs, transformer, spec, states}``; the
package is an UNPINNED dependency of the reference (``requirements.txt``: ``demucs``), not vendored
and not installed here, so the published demucs v4 (``htdemucs``) layers are restated from the
upstream algorithm: spectro / ispectro (normalized Hann STFT), pad1d, ScaledEmbedding, HEncLayer /
HDecLayer, DConv + LayerScale, rescale_module, capture_init, and the CrossTransformerEncoder
(sinusoidal 1-D / 2-D embeddings, norm-first self / cross attention layers with LayerScale and a
GroupNorm(1) output norm).  Parity at this boundary is UNPINNED (no reference test or fixture
covers it); everything in ``models/demucs4ht.py`` itself runs as the reference wrote it.
"""
