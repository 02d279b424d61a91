import ctypes, sys, torch
sys.path.insert(0, '/root/repo')
import __graft_entry__ as ge
pkg = ge.load_package()
loop = pkg.lib().hg_tune_launch_loop
loop.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
loop.restype = ctypes.c_double
dev = torch.device('cuda:0')
n = 1000
s = torch.rand(8, n, dtype=torch.float64, device=dev); t = torch.rand(8, n, dtype=torch.float64, device=dev); H = torch.empty(9, n, dtype=torch.float64, device=dev)
st = torch.cuda.current_stream().cuda_stream
for rep in range(3):
    print('empty', loop(2, 8, 0, 0, 0, 0, 1, 0, 20000, st), 'aca', loop(0, 8, s.data_ptr(), t.data_ptr(), H.data_ptr(), n, 1, 0, 20000, st),
          'aca-null-stream', loop(0, 8, s.data_ptr(), t.data_ptr(), H.data_ptr(), n, 1, 0, 20000, 0))
