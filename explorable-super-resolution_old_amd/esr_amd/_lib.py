"""ctypes binding of libesr_amd.so (C ABI declared in include/esr_amd.h).

The library is built in-tree (`make -C explorable-super-resolution_old_amd/csrc` or `__graft_entry__.build()`).  There
is no fallback: if the library cannot be loaded, or a caller hands it a non-ROCm tensor, we raise.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('ESR_AMD_LIB', os.path.join(_HERE, 'libesr_amd.so'))
ABI_VERSION = 23

c_int = ctypes.c_int32
c_float = ctypes.c_float
c_void_p = ctypes.c_void_p
c_fp = ctypes.POINTER(ctypes.c_float)


class ConvOut(ctypes.Structure):
    """Mirror of `esr_conv_out` (include/esr_amd.h)."""
    _fields_ = [('out', c_void_p),
                ('out_cp', c_int), ('out_coff', c_int), ('out_h', c_int), ('out_w', c_int),
                ('out_sy', c_int), ('out_sx', c_int), ('out_oy', c_int), ('out_ox', c_int), ('out_planar', c_int),
                ('lrelu', c_int),
                ('r1', c_void_p), ('r1_cp', c_int), ('r1_coff', c_int), ('s1', c_float),
                ('r2', c_void_p), ('r2_cp', c_int), ('r2_coff', c_int), ('s2', c_float),
                ('out2', c_void_p), ('out2_cp', c_int), ('out2_coff', c_int)]


class EsrOp(ctypes.Structure):
    """Mirror of `esr_op` (include/esr_amd.h): one recorded launch of an op list (esr_run_ops)."""
    _fields_ = [('kind', c_int), ('tag', c_int), ('p', c_void_p * 10), ('i', c_int * 20), ('f', c_float * 2),
                ('o', ConvOut)]


(OP_CONV3X3, OP_CONV3X3_X3, OP_UPCONV, OP_UPCONV_X3, OP_PREP, OP_CEM_DOWN, OP_CEM_INV, OP_CEM_UP_ADD, OP_HR_CONVS_X3,
 OP_HR1_SUM) = range(1, 11)

# name -> argtypes (all return int32 status unless listed in _RESTYPES)
_SIGNATURES = {
    'esr_conv3x3_fwd': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                        ctypes.POINTER(ConvOut), c_void_p],
    'esr_upconv2x_phase_fwd': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                               ctypes.POINTER(ConvOut), c_void_p],
    'esr_prep_input': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                       ctypes.POINTER(c_void_p), ctypes.POINTER(c_int), c_int,
                       ctypes.POINTER(c_void_p), ctypes.POINTER(c_int), c_int, c_int, c_void_p],
    'esr_conv3x3_fwd_x3': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_int,
                           ctypes.POINTER(ConvOut), c_void_p, c_void_p],
    'esr_upconv2x_phase_fwd_x3': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_int,
                                  c_int, c_int, ctypes.POINTER(ConvOut), c_void_p, c_void_p],
    'esr_hr_convs_x3': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                        c_void_p, c_void_p],
    'esr_hr1_sum': [c_void_p, c_int, c_int, c_int, c_void_p, c_float, c_void_p, c_void_p],
    'esr_cem_down': [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                     c_void_p],
    'esr_cem_inv': [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p],
    'esr_cem_up_add': [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int,
                       c_void_p],
    'esr_conv3x3_wgrad': [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                          c_void_p, c_void_p],
    'esr_wgrad_reduce': [c_void_p, c_int, ctypes.c_int64, c_float, c_void_p, c_void_p],
    'esr_bn_workspace_floats': [ctypes.c_int64, c_int],
    'esr_bn_lrelu_fwd': [c_void_p, ctypes.c_int64, c_int, c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_void_p],
    'esr_bn_lrelu_bwd': [c_void_p, c_void_p, ctypes.c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float,
                         c_void_p, c_void_p, c_void_p, c_void_p],
    'esr_bn_lrelu_bwd2': [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, ctypes.c_int64, c_int, c_void_p,
                          c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p],
    'esr_wgrad_reduce_gs': [c_void_p, c_int, ctypes.c_int64, c_float, c_void_p, c_void_p, c_void_p],
    'esr_wgrad_reduce2': [c_void_p, c_int, ctypes.c_int64, ctypes.c_int64, c_float, c_float, c_void_p, c_void_p,
                          c_void_p],
    'esr_prep_input_s': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                         ctypes.POINTER(c_void_p), ctypes.POINTER(c_int), c_int,
                         ctypes.POINTER(c_void_p), ctypes.POINTER(c_int), c_int, c_int, c_float, c_void_p],
    'esr_grad_amax': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    'esr_axpby_gs_amax': [c_void_p, c_int, c_int, c_float, c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_int,
                          c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    'esr_axpby_gs': [c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_int,
                     c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    'esr_lrelu_bwd': [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    'esr_lrelu_bwd_split': [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    'esr_axpby': [c_void_p, c_int, c_int, c_float, c_void_p, c_int, c_int, c_float, c_void_p, c_int, c_int, c_int,
                  c_int, c_int, c_int, c_void_p],
    'esr_sum2x2': [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    'esr_nchw_to_padded': [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p],
    'esr_cem_adjoint': [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                        c_float, c_int, c_void_p, c_void_p],
    'esr_input_adjoint': [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int,
                          c_int, c_void_p, c_void_p],
    'esr_dconv_fwd': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                      c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                      ctypes.POINTER(c_int), ctypes.POINTER(c_int), c_int, c_void_p],
    'esr_dconv_fwd_sk': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                         c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                         ctypes.POINTER(c_int), ctypes.POINTER(c_int), c_int, c_void_p, c_int, c_void_p],
    'esr_dconv_fwd_splits': [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_int),
                             ctypes.POINTER(c_int), c_int],
    'esr_dconv_fwd_sd': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
                         c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                         ctypes.POINTER(c_int), ctypes.POINTER(c_int), c_int, c_void_p, c_int, c_int, c_int, c_int,
                         c_int, c_void_p, c_void_p, c_void_p],
    'esr_dconv_uses_halo': [c_int, c_int, c_int, c_int, c_int, c_int],
    'esr_dconv_presplit': [c_void_p, ctypes.c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    'esr_colsum': [c_void_p, ctypes.c_int64, c_int, c_void_p, c_void_p, c_void_p],
    'esr_dfirst_fwd': [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_int, c_void_p, c_void_p,
                       c_void_p],
    'esr_dfirst_fwd_padded': [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_int, c_void_p,
                              c_int, c_int, c_void_p],
    'esr_dfirst_bwd_blocks': [c_int, c_int, c_int],
    'esr_dfirst_bwd': [c_void_p, c_void_p, c_void_p, c_float, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                       c_void_p],
    'esr_dconv_im2col': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    'esr_dconv_col2im': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    'esr_dconv_fwd_splits_sd': [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_int),
                                ctypes.POINTER(c_int), c_int, c_int],
    'esr_dconv_wgrad_splits': [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, ctypes.POINTER(c_int),
                               ctypes.POINTER(c_int), c_int],
    'esr_dconv_wgrad': [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int,
                        c_int, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int), c_int, c_void_p, c_int, c_void_p],
    'esr_timer_create': [c_int],
    'esr_timer_elapsed': [c_void_p, c_fp],
    'esr_timer_destroy': [c_void_p],
    'esr_timer_record': [c_void_p, c_int, c_void_p],
    'esr_timer_stamps': [c_void_p, c_void_p, c_fp],
    'esr_run_ops': [ctypes.POINTER(EsrOp), c_int, c_void_p, c_void_p],
    'esr_op_size': [],
    'esr_abi_version': [],
}
_RESTYPES = {'esr_timer_create': c_void_p, 'esr_timer_destroy': None, 'esr_bn_workspace_floats': ctypes.c_int64}
EXPORTED = tuple(_SIGNATURES)

# Extra entry points of the ABLATION library (csrc/esr_ablation.h; `make -C .../csrc exp` -> exp_lib/libesr_exp.so):
# process-wide kernel-selection setters for same-box A/B runs and the variant-equality tests.  The product library
# exports none of them (it has no selection state).
ABLATION_PATH = os.path.join(os.path.dirname(os.path.dirname(_HERE)), 'exp_lib', 'libesr_exp.so')
ABLATION_SETTERS = ('esr_x3_set_kernel', 'esr_x3_set_tile_map', 'esr_x3_set_narrow', 'esr_x3_set_nsplit',
                    'esr_conv_set_tile', 'esr_cem_set_direct', 'esr_wgrad_set_kernel', 'esr_wgrad3_set_dma',
                    'esr_dconv_set_halo', 'esr_dconv_set_occ3', 'esr_dconv_set_cw16', 'esr_dconv_set_rows',
                    'esr_axpby_set_rows', 'esr_bn_set_onepass', 'esr_x3c_set_stamps', 'esr_wgrad3d_set_dbg',
                    'esr_wgrad3d_set_unroll')

_lib = None


class ESRLibraryError(RuntimeError):
    pass


def bind(path):
    """ctypes handle of the library at `path` with every prototype bound (the product ABI, plus the ablation setters
    when the library exports them).  Raises ESRLibraryError if absent or ABI-incompatible."""
    if not os.path.exists(path):
        raise ESRLibraryError('%s not found: build it with `make -C explorable-super-resolution_old_amd/csrc` (or '
                              '__graft_entry__.build()); there is no non-HIP fallback' % path)
    lib = ctypes.CDLL(path)
    for name, argtypes in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPES.get(name, c_int)
    v = lib.esr_abi_version()
    if v != ABI_VERSION:
        raise ESRLibraryError('%s ABI %d != expected %d (stale build?)' % (path, v, ABI_VERSION))
    if lib.esr_op_size() != ctypes.sizeof(EsrOp):
        raise ESRLibraryError('esr_op layout mismatch: C %d bytes, binding %d' % (lib.esr_op_size(),
                                                                                  ctypes.sizeof(EsrOp)))
    if hasattr(lib, 'esr_x3_set_kernel'):  # the ablation library
        for name in ABLATION_SETTERS:
            fn = getattr(lib, name)
            fn.argtypes = [c_void_p] if name == 'esr_x3c_set_stamps' else [c_int]  # (a stamp buffer; the rest: ints)
            fn.restype = c_int
        # same-box A/B runs of whole benchmarks (tools/gpu_ab_env.sh with ESR_AMD_LIB=exp_lib/libesr_exp.so)
        if os.environ.get('ESR_X3_NSPLIT') in ('0', '1'):
            lib.esr_x3_set_nsplit(int(os.environ['ESR_X3_NSPLIT']))
        if os.environ.get('ESR_AXPBY_ROWS') in ('0', '1'):
            lib.esr_axpby_set_rows(int(os.environ['ESR_AXPBY_ROWS']))
        if os.environ.get('ESR_X3_KERNEL', '').isdigit():
            lib.esr_x3_set_kernel(int(os.environ['ESR_X3_KERNEL']))
        if os.environ.get('ESR_WGRAD3D_UNROLL') in ('1', '2', '4'):
            lib.esr_wgrad3d_set_unroll(int(os.environ['ESR_WGRAD3D_UNROLL']))
    else:
        stale = [k for k in RETIRED_ENV if k in os.environ]
        if stale:  # switches of earlier rounds: the product library has no selection state, so they change nothing
            import warnings
            warnings.warn('esr_amd: %s set but %s is the product library, which has no kernel-selection state: '
                          'the default kernels run; for an A/B use the ablation library (ESR_AMD_LIB=%s)'
                          % (', '.join(stale), os.path.basename(path), ABLATION_PATH), RuntimeWarning, stacklevel=2)
    return lib


# environment switches that now act only through the ablation library's setters (ignored by the product library)
RETIRED_ENV = ('ESR_X3_NSPLIT', 'ESR_AXPBY_ROWS', 'ESR_X3_KERNEL', 'ESR_WGRAD3D_UNROLL', 'ESR_DCONV_HALO',
               'ESR_DCONV_OCC3', 'ESR_DCONV_CW16', 'ESR_DCONV_ROWS', 'ESR_WGRAD3_DMA', 'ESR_X3_TILE_MAP', 'ESR_X3_NARROW')


def load():
    """The library of the product path (libesr_amd.so, or ESR_AMD_LIB), loaded once."""
    global _lib
    if _lib is None:
        _lib = bind(LIB_PATH)
    return _lib


_ablation = None


def load_ablation():
    """The ablation library (exp_lib/libesr_exp.so), loaded once; ESRLibraryError if it was not built."""
    global _ablation
    if _ablation is None:
        _ablation = bind(ABLATION_PATH)
    return _ablation


def check(rc, what):
    if rc != 0:
        raise RuntimeError('%s failed with esr_status %d' % (what, rc))


def ptr(t):
    """Device pointer of a tensor (None → NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())
