import ctypes, os, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libmfmapeak.so'))
out = torch.zeros(512, device='cuda')
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for blocks in (256, 512, 1536):
    iters = 4000
    lib.run_peak(ctypes.c_void_p(out.data_ptr()), blocks, iters, st)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(); lib.run_peak(ctypes.c_void_p(out.data_ptr()), blocks, iters, st); e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e)
    flop = blocks * 8 * iters * 4 * 2 * 32 * 32 * 16
    print('blocks %d: %.3f ms  %.1f TFLOP/s f16' % (blocks, ms, flop / ms / 1e9))
