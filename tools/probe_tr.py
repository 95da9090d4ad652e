import ctypes, os, torch
torch.cuda.init()
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprobe_tr.so"))
src = (torch.arange(64 * 64, dtype=torch.int32) // 64 * 256 + torch.arange(64 * 64, dtype=torch.int32) % 64).to(torch.int16).cuda()
for mode in range(4):
    out = torch.zeros(256, dtype=torch.int32, device="cuda")
    rc = lib.probe(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(out.data_ptr()), mode)
    o = out.cpu().view(64, 4).tolist()
    print("mode", mode, "rc", rc)
    for l in [0, 1, 4, 5, 16, 17, 32, 48]:
        print("  lane", l, [(v // 256, v % 256) for v in o[l]])
