"""First-touch cost of a fresh 1.6 GB host matrix (what R's allocMatrix hands the library): 8
threads writing it, with and without madvise(MADV_HUGEPAGE) on the range first."""
import ctypes
import mmap
import threading
import time

import numpy as np

libc = ctypes.CDLL("libc.so.6", use_errno=True)
MADV_HUGEPAGE = 14
for p in ("/sys/kernel/mm/transparent_hugepage/enabled", "/sys/kernel/mm/transparent_hugepage/defrag"):
    try:
        print(p, open(p).read().strip())
    except OSError as e:
        print(p, e)


def touch(buf, nthreads=8):
    n = len(buf)
    def work(i):
        a, z = n * i // nthreads, n * (i + 1) // nthreads
        buf[a:z] = 1.0
    ts = [threading.Thread(target=work, args=(i,)) for i in range(nthreads)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return (time.perf_counter() - t0) * 1e3


N = 200_000_000
for rep in range(3):
    for huge in (False, True):
        m = mmap.mmap(-1, 8 * N, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        addr = ctypes.addressof(ctypes.c_char.from_buffer(m))
        if huge:
            al = (addr + (1 << 21) - 1) & ~((1 << 21) - 1)
            r = libc.madvise(ctypes.c_void_p(al), ctypes.c_size_t(8 * N - (al - addr)), MADV_HUGEPAGE)
        buf = np.frombuffer(m, dtype=np.float64)
        ms = touch(buf)
        ms2 = touch(buf)
        print(f"rep {rep} huge {huge}: first touch {ms:.1f} ms, again {ms2:.1f} ms", flush=True)
        del buf
        m.close()
