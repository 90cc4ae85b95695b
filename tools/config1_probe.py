"""BASELINE config 1 end to end: `xspect classify species` on one assembly
FASTA, as a user runs it (one process per call), through this package's
classify.classify_species (classify.py; reference src/xspect/classify.py:43-92).

Setup (a child process): a 100-species model fitted on the GPU from seeded
4 Mbp genomes (one FASTA per species, as the reference trains from a
directory), saved under a temporary XSPECT_DATA; an assembly of one species
(4 Mbp in 3 contigs, 80-column FASTA).  Then --reps fresh processes each run
classify_species on it; each reports the phases (imports, model load, predict,
save) and its wall time; the parent adds the time of the whole child process.
One JSON line.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

SETUP = r"""
import sys
sys.path.insert(0, %r)
from pathlib import Path
from xspect2_amd.file_io import Record, write_fasta
from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel
from xspect2_amd.synth import make_genomes
root = Path(%r)
g = make_genomes(100, 4_000_000, seed=7)
sp = root / "species"
sp.mkdir(parents=True, exist_ok=True)
for i in range(100):
    write_fasta([Record(f"c{i}", g[i].tobytes().decode())], sp / f"GCF_{i:09d}.1_X_genomic.fna", width=80)
m = ProbabilisticFilterModel(21, "Acinetobacter", None, None, "Species", root / "xspect-data" / "models")
m.fit(sp)
m.save()
a = g[42].tobytes().decode()
write_fasta([Record("contig_1", a[:1_500_000]), Record("contig_2", a[1_500_000:3_000_000]),
             Record("contig_3", a[3_000_000:])], root / "assembly.fna", width=80)
"""

RUN = r"""
import sys, time, json
t0 = time.perf_counter()
sys.path.insert(0, %r)
from xspect2_amd import classify
from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel
t = {"imports_s": time.perf_counter() - t0}
from pathlib import Path
root = Path(%r)
t1 = time.perf_counter()
m = ProbabilisticFilterModel.load(classify.species_model_path("Acinetobacter"))
t["model_load_s"] = time.perf_counter() - t1
t1 = time.perf_counter()
r = m.predict_columnar(root / "assembly.fna")
t["predict_s"] = time.perf_counter() - t1
r.input_source = "assembly.fna"
t1 = time.perf_counter()
r.save(root / "out.json")
t["save_s"] = time.perf_counter() - t1
m.close()
t1 = time.perf_counter()
classify.classify_species("Acinetobacter", root / "assembly.fna", root / "out2.json")
t["classify_species_again_s"] = time.perf_counter() - t1
t["total_s"] = time.perf_counter() - t0
t["same_json"] = (root / "out.json").read_bytes() == (root / "out2.json").read_bytes()
print(json.dumps(t))
"""


def main():
    reps = 3
    root = Path(tempfile.mkdtemp(prefix="xs_config1_"))
    env = dict(os.environ, XSPECT_DATA=str(root / "xspect-data"))
    t = time.perf_counter()
    subprocess.run([sys.executable, "-c", SETUP % (str(ROOT), str(root))], check=True, env=env)
    setup_s = time.perf_counter() - t
    runs = []
    for _ in range(reps):
        t = time.perf_counter()
        r = subprocess.run([sys.executable, "-c", RUN % (str(ROOT), str(root))], check=True, env=env,
                           capture_output=True, text=True)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        d["process_s"] = time.perf_counter() - t
        runs.append(d)
    import shutil
    shutil.rmtree(root)
    print(json.dumps({"setup_s": setup_s, "runs": runs,
                      "best_process_s": min(r["process_s"] for r in runs)}), flush=True)


if __name__ == "__main__":
    main()
