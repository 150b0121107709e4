"""What the HIP runtime reports for a hipHostRegister'ed (mapped) numpy buffer
versus a hipHostMalloc one: the pointer attributes and address ranges
host.hip's direct mode relies on.  Prints one JSON line."""
import ctypes as C
import json

import numpy as np
import torch

hip = C.CDLL("libamdhip64.so")
torch.cuda.init()


class Attr(C.Structure):  # hipPointerAttribute_t (type, device, devicePointer, hostPointer, isManaged, allocationFlags)
    _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p), ("hostPointer", C.c_void_p),
                ("isManaged", C.c_int), ("allocationFlags", C.c_uint)]


def probe(ptr, nbytes):
    out = {}
    a = Attr()
    out["getAttributes"] = hip.hipPointerGetAttributes(C.byref(a), C.c_void_p(ptr))
    out["type"] = a.type
    d = C.c_void_p()
    out["getDevicePointer"] = hip.hipHostGetDevicePointer(C.byref(d), C.c_void_p(ptr), 0)
    out["dev_eq_host"] = d.value == ptr
    for name, q in (("dev", d.value), ("host", ptr)):
        base, size = C.c_void_p(), C.c_size_t()
        rc = hip.hipMemGetAddressRange(C.byref(base), C.byref(size), C.c_void_p(q))
        out[f"range_{name}"] = [rc, (base.value or 0) - (q or 0), size.value]
        rs = hip.hipPointerGetAttribute(C.byref(base), 11, C.c_void_p(q))  # RANGE_START_ADDR
        rz = hip.hipPointerGetAttribute(C.byref(size), 12, C.c_void_p(q))  # RANGE_SIZE
        out[f"attr_range_{name}"] = [rs, rz, (base.value or 0) - (q or 0), size.value]
    hip.hipGetLastError()
    return out


n = 1 << 20
raw = np.zeros(n + 8192, np.uint8)
off = (-raw.ctypes.data) % 4096
buf = raw[off:off + n]
res = {"register_rc": hip.hipHostRegister(C.c_void_p(buf.ctypes.data), C.c_size_t(n), 2)}
res["registered"] = probe(buf.ctypes.data, n)
res["registered_mid"] = probe(buf.ctypes.data + 4096, n - 4096)
hip.hipHostUnregister(C.c_void_p(buf.ctypes.data))
p = C.c_void_p()
hip.hipHostMalloc(C.byref(p), C.c_size_t(n), 0)
res["hostmalloc"] = probe(p.value, n)
hip.hipHostFree(p)
print(json.dumps(res))
