"""CPU oracle for the chunk-reduction hot path — TEST INFRASTRUCTURE ONLY.

Nothing in ``pyactivestorage_amd`` imports this package. Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
use it, and only as the checker / the timed CPU baseline, never as the thing
that is measured or shipped.

Pinning: ``storage_ref`` is checked against golden vectors produced by running
the reference's own ``activestorage/storage.py`` (loaded by file path in the
build container, see ``tests/golden/make_golden.py``) and against the
known answers hard-coded in the reference's tests (``tests/golden/known_answers.json``).
"""
