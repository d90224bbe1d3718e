import ctypes, os, sys, subprocess
mode = sys.argv[1]
if mode == "torch":
    import torch
    x = torch.zeros(1, device="cuda")
    lib = ctypes.CDLL(sys.argv[2])
    for l in open("/proc/self/maps"):
        if "amdhip64" in l:
            print("maps:", l.split()[-1]); 
    aa = torch.tensor([[0.1, 0.2, 0.3]] * 4, device="cuda")
    R = torch.empty(4, 3, 3, device="cuda")
    lib.tik_last_error.restype = ctypes.c_char_p
    s = torch.cuda.current_stream().cuda_stream
    print("stream", s)
    rc = lib.tik_aa_to_rotmat(ctypes.c_void_p(aa.data_ptr()), 4, ctypes.c_void_p(R.data_ptr()), ctypes.c_void_p(s))
    print(mode, sys.argv[2], "rc", rc, lib.tik_last_error())
    torch.cuda.synchronize(); print(R[0])
