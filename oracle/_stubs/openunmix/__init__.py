"""openunmix placeholder.  TEST INFRASTRUCTURE ONLY: models/demucs4ht.py:14 imports
``openunmix.filtering.wiener`` at module scope; it is only called when ``cac`` is False and
``wiener_iters >= 0`` (demucs4ht.py:472-478), which the released HTDemucs configs never select."""
