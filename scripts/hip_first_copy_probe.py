"""Which HIP call pays the runtime's lazy initialisation in a fresh process
(GPU box): device count, hipMalloc, hipHostMalloc, a copy from pinned memory,
a copy from pageable memory, hipMemset, in that order (or the order given as
argv). usage: python3 scripts/hip_first_copy_probe.py [order]"""
import ctypes as C
import sys
import time

hip = C.CDLL("libamdhip64.so")
n = C.c_int(0)
t = time.perf_counter()
hip.hipGetDeviceCount(C.byref(n))
print("device count %8.3f ms" % ((time.perf_counter() - t) * 1e3))
d = C.c_void_p()
h = C.c_void_p()
page = (C.c_char * 4096)()
steps = {
    "malloc": lambda: hip.hipMalloc(C.byref(d), C.c_size_t(4096)),
    "hostmalloc": lambda: hip.hipHostMalloc(C.byref(h), C.c_size_t(4096), C.c_uint(0)),
    "copy_pinned": lambda: hip.hipMemcpy(d, h, C.c_size_t(4096), C.c_int(1)),
    "copy_pageable": lambda: hip.hipMemcpy(d, page, C.c_size_t(4096), C.c_int(1)),
    "memset": lambda: hip.hipMemset(d, C.c_int(0), C.c_size_t(4096)),
    "copy_d2h_pinned": lambda: hip.hipMemcpy(h, d, C.c_size_t(4096), C.c_int(2)),
}
order = sys.argv[1].split(",") if len(sys.argv) > 1 else ["malloc", "hostmalloc", "copy_pinned", "copy_pageable", "memset",
                                                          "copy_d2h_pinned"]
for s in order:
    t = time.perf_counter()
    rc = steps[s]()
    print("%-16s %8.3f ms rc %d" % (s, (time.perf_counter() - t) * 1e3, rc))
