"""ctypes signatures of the C ABI exported by ``_zkamd.so``.

Kept next to the loader so the Python and C++ sides can be checked against
each other (``tests/test_native_abi.py`` compares this table with the symbols
of the built library)."""

import ctypes as C

P = C.c_void_p
I32 = C.c_int
I64 = C.c_int64
F32 = C.c_float

U64 = C.c_uint64
FP = C.POINTER(C.c_float)

SIGNATURES = {
    # host runtime
    "zk_gather_rows": (I32, [P, I64, P, I64, P, I32]),
    # preprocessing
    "zk_normalize_flip_c3": (I32, [P, P, I32, I32, I32, FP, FP, I32, U64, P]),
    # optimizers
    "zk_adam_step": (I32, [P, P, P, P, P, I32, F32, F32, F32, F32, F32, F32, F32, F32, P]),
    "zk_sgd_step": (I32, [P, P, P, P, I32, F32, F32, F32, F32, I32, P]),
}
