"""MI355X (gfx950) chunk-reduction backend for PyActiveStorage.

Drop-in for ``activestorage/storage.py``'s local ``reduce_chunk`` (see
``pyactivestorage_amd.storage``) plus a batched, device-resident engine for
whole queries (``pyactivestorage_amd.active`` / ``.batch``).  Native code:
``pyactivestorage_amd/csrc`` (HIP) behind the C ABI in ``include/pyas.h``.
"""
__version__ = "0.1.0"
