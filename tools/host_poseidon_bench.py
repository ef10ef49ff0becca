"""Host Poseidon absorb timing through the C-ABI (tpst_transcript_append_bytes)."""
import ctypes as C, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from testudo_amd import _lib
lib = _lib.load()
st = C.create_string_buffer(4096)
lib.tpst_transcript_init(st)
buf = bytes(list(range(256)) * 2 + list(range(64)))
for _ in range(20): lib.tpst_transcript_append_bytes(st, buf, 576)
t = time.perf_counter(); N = 400
for _ in range(N): lib.tpst_transcript_append_bytes(st, buf, 576)
dt = (time.perf_counter() - t) / N
print("append 576 B: %.1f us (%.2f us per permutation)" % (dt * 1e6, dt * 1e6 / 6.5))
out = (C.c_uint64 * 4)()
lib.tpst_transcript_challenge(st, out); print([hex(x) for x in out])
