"""Debug: one resident-mode decode case (RLE_MI355X_SEG_RES=1), first mismatches."""
import os, sys
R_ = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R_, "c-filestorage-server-and-client_amd"), os.path.join(R_, "oracle"), os.path.join(R_, "tests")]
import rle_oracle as O
from test_gpu_parity import gpu_decode, gpu_encode
for (kind, seed, U) in [(2, 106, 7055), (2, 106, 7057), (2, 106, 3000), (1, 5, 8047), (2, 7, 20000), (0, 1, 30000), (3, 3, 30000), (2, 9, 60000)]:
    x = O.gen(kind, seed, U)
    y = O.encode(x)
    dec, st = gpu_decode([y], [len(x)], seg=True)
    d = dec[0]
    bad = [i for i in range(len(x)) if d[i] != x[i]]
    print(kind, seed, U, "C", len(y), "status", st[0], "nbad", len(bad), "first", bad[:8], "last", bad[-3:], flush=True)
    if bad:
        i = bad[0]
        print("   got", d[i-4:i+12].hex(), "\n   exp", x[i-4:i+12].hex())
