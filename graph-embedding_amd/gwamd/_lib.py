"""ctypes binding of libgraphwalk (include/graphwalk.h).

The shared library is built in-tree by graph-embedding_amd/build.py.  There is
no CPU fallback: if the library (or a GPU, for compute calls) is missing the
calls raise.

torch is imported first when it is installed: libtorch ships its own
libamdhip64.so.7, and loading it before libgraphwalk makes both share ONE HIP
runtime (so torch streams/pointers are valid handles for this library).
"""
import ctypes
import os

try:  # share torch's HIP runtime (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the library
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GW_LIB", os.path.join(_HERE, "libgraphwalk.so"))

GW_OK = 0
GW_ERR_INVALID = -1
GW_ERR_IO = -2
GW_ERR_PARSE = -3
GW_ERR_NOMEM = -4
GW_ERR_DEVICE = -5
GW_ERR_STATE = -6
GW_ERR_UNSUPPORTED = -7
GW_ERR_RANGE = -8
GW_ERR_KEY = -9
GW_ERR_ZERODIV = -10
GW_ERR_CAPACITY = -11

SEM_NX_SIMPLE = 0
SEM_JAVA_MULTI = 1
N2V_REPLAY = 0
N2V_REJECTION = 1
N2V_BITSET = 2
N2V_AUTO = 3
TOPSIM_SINGLE_SAMPLE = 0
TOPSIM_ENUMERATE = 1
TOPSIM_SINGLE_RW = 2
DOUBLE_SAMPLE = 0
DOUBLE_DEV = 1
DOUBLE_RANDOM_WALK = 2


class GraphWalkError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class DeviceError(GraphWalkError):
    pass


class CapacityError(GraphWalkError):
    pass


class StateError(GraphWalkError):
    pass


class UnsupportedError(GraphWalkError):
    pass


class GraphInfo(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("nnz", ctypes.c_int64),
                ("max_degree", ctypes.c_int64), ("edge_alias_entries", ctypes.c_int64),
                ("semantics", ctypes.c_int32), ("directed", ctypes.c_int32),
                ("weighted", ctypes.c_int32), ("device", ctypes.c_int32),
                ("sampler_bytes", ctypes.c_int64), ("n2v_mode", ctypes.c_int32), ("listed", ctypes.c_int32)]


class Options(ctypes.Structure):
    """gw_options_t (per-handle tuning, include/graphwalk.h)."""
    _fields_ = [("table_budget_bytes", ctypes.c_int64), ("expected_steps", ctypes.c_int64),
                ("listed", ctypes.c_int32), ("simrank_hbm_row", ctypes.c_int32),
                ("host_chunk_bytes", ctypes.c_int64), ("topsim_part_shrink", ctypes.c_int32),
                ("reserved0", ctypes.c_int32)]


P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
D = ctypes.c_double
CP = ctypes.c_char_p
PI32 = ctypes.POINTER(ctypes.c_int32)
PI64 = ctypes.POINTER(ctypes.c_int64)
PD = ctypes.POINTER(ctypes.c_double)
PP = ctypes.POINTER(ctypes.c_void_p)

# name -> (restype, argtypes); mirrors include/graphwalk.h one to one
SIGNATURES = {
    "gw_version": (CP, []),
    "gw_last_error": (CP, [P]),
    "gw_strerror": (CP, [ctypes.c_int]),
    "gw_device_count": (ctypes.c_int, [PI32]),
    "gw_philox4x32": (ctypes.c_int, [ctypes.c_int, P, I64, P]),
    "gw_graph_load_edgelist": (ctypes.c_int, [CP, CP, ctypes.c_int, ctypes.c_int, ctypes.c_int, I64, PP]),
    "gw_graph_from_edges": (ctypes.c_int, [I64, P, P, P, ctypes.c_int, ctypes.c_int, I64, PP]),
    "gw_graph_from_csr": (ctypes.c_int, [I64, P, P, P, P, P, ctypes.c_int, ctypes.c_int, PP]),
    "gw_graph_rmat": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, D, D, D, U64, PP]),
    "gw_graph_rmat_java": (ctypes.c_int, [I64, I64, D, D, D, U64, PP]),
    "gw_graph_info": (ctypes.c_int, [P, ctypes.POINTER(GraphInfo)]),
    "gw_graph_set_options": (ctypes.c_int, [P, ctypes.POINTER(Options)]),
    "gw_graph_get_options": (ctypes.c_int, [P, ctypes.POINTER(Options)]),
    "gw_graph_export_csr": (ctypes.c_int, [P, P, P, P, P, P]),
    "gw_graph_free": (ctypes.c_int, [P]),
    "gw_graph_to_device": (ctypes.c_int, [P, ctypes.c_int]),
    "gw_n2v_prepare": (ctypes.c_int, [P, D, D, ctypes.c_int]),
    "gw_n2v_export_alias": (ctypes.c_int, [P, P, P, P, P, P]),
    "gw_alias_setup": (ctypes.c_int, [ctypes.c_int, P, I64, P, P]),
    "gw_n2v_walks_replay": (ctypes.c_int, [P, ctypes.c_int, I64, P, P, I64, P, P, PI64]),
    "gw_n2v_walks": (ctypes.c_int, [P, ctypes.c_int, U64, I64, I64, ctypes.c_int, P, P, P, P]),
    "gw_n2v_walks_host": (ctypes.c_int, [P, ctypes.c_int, U64, I64, I64, ctypes.c_int, P, P, P]),
    "gw_topsim_host": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, D, U64, P, I64,
                                      ctypes.c_int, P, P, P, P]),
    "gw_topsim_prepare":(ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "gw_topsim_kernel": (ctypes.c_char_p, [P]),
    "gw_topsim_kernel_attrs": (ctypes.c_int, [P, P, P, P]),
    "gw_topsim": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, D, U64, P, I64,
                                 ctypes.c_int, P, P, P, P]),
    "gw_topsim_dense": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, D, U64, P, I64,
                                       P, P, P]),
    "gw_topsim_sparse": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, D, U64, P, I64, I64,
                                        P, P, P, P, P, P, P]),
    "gw_topsim_write_text": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, D, U64, P, I64,
                                            ctypes.c_int, CP, CP, ctypes.c_int, P]),
    "gw_topsim_m": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, D, U64, P, I64,
                                   P, P, P, P, P]),
    "gw_topsim_m_host": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, D, U64, P,
                                        I64, P, P, P, P]),
    "gw_topsim_double": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, D, U64, P, P]),
    "gw_topsim_dev": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, D, U64, P, P, P]),
    "gw_double_random_walk": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, D, U64, P, P]),
    "gw_double_sim_host": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          D, U64, P, P]),
    "gw_select_fixed_max_pq": (ctypes.c_int, [P, I64, I64, ctypes.c_int, D, P]),
    "gw_format_java_double": (ctypes.c_int, [D, ctypes.c_char_p, I64]),
    "gw_simrank_naive": (ctypes.c_int, [P, D, ctypes.c_int, P, P]),
    "gw_simrank_naive_host": (ctypes.c_int, [P, D, ctypes.c_int, P]),
    "gw_write_walks_text": (ctypes.c_int, [P, CP, P, P, I64, ctypes.c_int]),
    "gw_write_sim_text_dense": (ctypes.c_int, [CP, P, P, I64, I64, ctypes.c_int, CP, ctypes.c_int]),
    "gw_write_sim_text_topk": (ctypes.c_int, [CP, P, P, P, I64, ctypes.c_int, CP, ctypes.c_int]),
    "gw_write_sim_text_sparse": (ctypes.c_int, [CP, P, P, P, P, P, I64, I64, ctypes.c_int, CP, ctypes.c_int]),
    "gw_write_sim_text_cachemap": (ctypes.c_int, [CP, P, P, P, P, I64, ctypes.c_int, ctypes.c_int, CP]),
    "gw_comm_unique_id": (ctypes.c_int, [P]),
    "gw_comm_init": (ctypes.c_int, [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, PP]),
    "gw_comm_allgather": (ctypes.c_int, [P, P, P, I64, ctypes.c_int, P]),
    "gw_comm_free": (ctypes.c_int, [P]),
    "gw_comm_last_error": (CP, [P]),
}

_lib = None


def lib():
    """Load libgraphwalk.so (raises ImportError when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libgraphwalk.so not found at {LIB_PATH}: run `python graph-embedding_amd/build.py` "
                "(there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc, handle=None):
    if rc == GW_OK:
        return
    L = lib()
    msg = L.gw_last_error(handle).decode(errors="replace")
    if rc == GW_ERR_INVALID:
        raise ValueError(msg)
    if rc == GW_ERR_IO:
        raise OSError(msg)
    if rc in (GW_ERR_PARSE,):
        raise ValueError(f"parse error: {msg}")
    if rc == GW_ERR_NOMEM:
        raise MemoryError(msg)
    if rc == GW_ERR_DEVICE:
        raise DeviceError(rc, msg)
    if rc == GW_ERR_STATE:
        raise StateError(rc, msg)
    if rc == GW_ERR_UNSUPPORTED:
        raise UnsupportedError(rc, msg)
    if rc == GW_ERR_RANGE:
        raise IndexError(msg)
    if rc == GW_ERR_KEY:
        raise KeyError(msg)
    if rc == GW_ERR_ZERODIV:
        raise ZeroDivisionError(msg)
    if rc == GW_ERR_CAPACITY:
        raise CapacityError(rc, msg)
    raise GraphWalkError(rc, msg)


def ptr(a):
    """Raw address of a numpy array / torch tensor / None."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    return ctypes.c_void_p(a.ctypes.data)


def device_count():
    c = ctypes.c_int32(0)
    rc = lib().gw_device_count(ctypes.byref(c))
    return c.value if rc == GW_OK else 0
