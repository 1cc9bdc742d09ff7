"""Probe (diagnostic): stream memory operations on this box -- hipExtMallocWithFlags(hipMallocSignalMemory),
hipStreamWriteValue32 / hipStreamWaitValue32 between two streams -- return codes and timing."""
import ctypes as C
import time

hip = C.CDLL("/opt/rocm/lib/libamdhip64.so")
hip.hipGetErrorString.restype = C.c_char_p


def chk(name, rc):
    print(name, rc, hip.hipGetErrorString(rc).decode(), flush=True)
    return rc


chk("hipSetDevice", hip.hipSetDevice(0))
ok = C.c_int(0)
chk("attr CanUseStreamWaitValue", hip.hipDeviceGetAttribute(C.byref(ok), 76 if False else C.c_int(0), 0) if False else 0)
p = C.c_void_p()
chk("hipExtMallocWithFlags signal", hip.hipExtMallocWithFlags(C.byref(p), C.c_size_t(64), C.c_uint(2)))
print("ptr", p.value)
chk("hipMemset", hip.hipMemset(p, 0, C.c_size_t(64)))
s1, s2 = C.c_void_p(), C.c_void_p()
chk("stream1", hip.hipStreamCreateWithFlags(C.byref(s1), 1))
chk("stream2", hip.hipStreamCreateWithFlags(C.byref(s2), 1))
chk("write32", hip.hipStreamWriteValue32(s1, p, C.c_uint32(5), C.c_uint(0)))
chk("wait32", hip.hipStreamWaitValue32(s2, p, C.c_uint32(5), C.c_uint(1), C.c_uint32(0xffffffff)))
t0 = time.perf_counter()
chk("sync2", hip.hipStreamSynchronize(s2))
print("waited", time.perf_counter() - t0)
chk("last", hip.hipGetLastError())
# device memory (plain hipMalloc) as the signal word
q = C.c_void_p()
chk("hipMalloc", hip.hipMalloc(C.byref(q), C.c_size_t(64)))
chk("write32 dev", hip.hipStreamWriteValue32(s1, q, C.c_uint32(7), C.c_uint(0)))
chk("wait32 dev", hip.hipStreamWaitValue32(s2, q, C.c_uint32(7), C.c_uint(1), C.c_uint32(0xffffffff)))
chk("sync2 dev", hip.hipStreamSynchronize(s2))
chk("last", hip.hipGetLastError())
