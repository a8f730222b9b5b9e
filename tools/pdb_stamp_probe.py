"""Per-phase k_pdb_scan times per file (largest six) from ab/pdbstamp/libpst.so (tools/pdb_stamps_build.py)
(PST_LIB=<that lib>): python tools/pdb_stamp_probe.py"""
import ctypes, json, os, sys, tarfile, tempfile
import numpy as np
ROOT = "/root/repo"
sys.path.insert(0, os.path.join(ROOT, "protein-structure-tokenizer_amd"))
import torch  # noqa
from pst_amd import params as P
from pst_amd._native import Tokenizer, LIB_PATH
with tempfile.TemporaryDirectory(dir="/dev/shm") as d:
    with tarfile.open(os.path.join(ROOT, "tests", "golden", "casp14_pdbs.tar.gz")) as tf:
        tf.extractall(d, members=[m for m in tf.getmembers() if m.isfile() and m.name.endswith(".pdb")])
    files = sorted(os.path.join(d, "casp14_pdbs", f) for f in os.listdir(os.path.join(d, "casp14_pdbs")))
    tk = Tokenizer(0, 4096, 1, P.random_blob(6, 1234))
    for _ in range(5):
        tk.tokenize_pdb_files(files, n_threads=16)
    L = ctypes.CDLL(LIB_PATH)
    st = np.zeros(64 * 16, np.uint64)
    L.pst_x_pdb_stamps(st.ctypes.data_as(ctypes.c_void_p))
    st = st.reshape(64, 16).astype(np.int64)
    sizes = [os.path.getsize(f) for f in files]
    t0 = st[:len(files), 0].min()
    rows = []
    for f in range(len(files)):
        s = st[f]
        ph = [(s[k + 1] - s[k]) / 100.0 for k in range(8)]  # us (100 MHz)
        rows.append({"file": os.path.basename(files[f]), "bytes": sizes[f], "start_us": (s[0] - t0) / 100.0,
                     "phases_us": ph, "total_us": (s[8] - s[0]) / 100.0})
    rows.sort(key=lambda r: -r["bytes"])
    for r in rows[:6]:
        print(json.dumps(r))
    print("phases: 0 lines (+ kinds), 1 kinds pass (gone: ~0), 2 stop, 3 records, 4 runs, 5 run loop+slot init, 6 atom slots, 7 kept scan")
