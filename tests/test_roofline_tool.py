"""tools/roofline_pmc.py, the per-ray PMC table bench.py's roofline reads: the
clock pass (GRBM_GUI_ACTIVE summed over the 8 XCDs / 8 / the dispatch's ns,
MI355X_MICROARCH.md "DVFS give-back") and the --clock-only merge into an
existing record, on a synthetic rocprofv3 counter CSV (no GPU)."""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = ('"Correlation_Id","Dispatch_Id","Agent_Id","Queue_Id","Process_Id","Thread_Id","Grid_Size","Kernel_Id",'
          '"Kernel_Name","Workgroup_Size","LDS_Block_Size","Scratch_Size","VGPR_Count","Accum_VGPR_Count",'
          '"SGPR_Count","Counter_Name","Counter_Value","Start_Timestamp","End_Timestamp"')


def counter_dir(path, rows):
    os.makedirs(path)
    with open(os.path.join(path, "run_counter_collection.csv"), "w") as f:
        f.write(HEADER + "\n")
        for did, name, counter, value, t0, t1 in rows:
            f.write(f'{did},{did},"Agent 2",1,1,1,512,6,"{name}",256,0,0,8,0,32,"{counter}",{value},{t0},{t1}\n')
    return path


def test_clock_only_merges_last_megakernel(tmp_path):
    out = tmp_path / "roofline_pmc.json"
    shutil.copy(os.path.join(ROOT, "profiles", "roofline_pmc.json"), out)
    d = counter_dir(str(tmp_path / "clk"), [
        (1, "film_reduce", "GRBM_GUI_ACTIVE", 1.0e6, 0, 10 ** 6),                    # not the megakernel
        (2, "path_megakernel<8, 4>", "GRBM_GUI_ACTIVE", 3.2e9, 10 ** 9, 10 ** 9 + 2 * 10 ** 8),
        (2, "path_megakernel<8, 4>", "GRBM_COUNT", 3.2e9, 10 ** 9, 10 ** 9 + 2 * 10 ** 8),
        (3, "path_megakernel<8, 4>", "GRBM_GUI_ACTIVE", 3.6e9, 2 * 10 ** 9, 2 * 10 ** 9 + 2 * 10 ** 8),
        (3, "path_megakernel<8, 4>", "GRBM_COUNT", 3.6e9, 2 * 10 ** 9, 2 * 10 ** 9 + 2 * 10 ** 8),
    ])
    key = "path:cornell:1920x1080"
    before = json.load(open(out))[key]
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline_pmc.py"), key, "--clock", d,
                    "--clock-only", "--out", str(out)], check=True, capture_output=True)
    rec = json.load(open(out))[key]
    assert abs(rec["clock_ghz"] - 3.6e9 / 8 / 2e8) < 1e-9          # the last dispatch: 2.25 GHz
    assert abs(rec["clock_dispatch_ms"] - 200.0) < 1e-9
    assert rec["valu_insts_per_ray"] == before["valu_insts_per_ray"]   # the rest of the record kept
    assert rec["source"].startswith(before["source"].split(", " + d)[0]) and rec["source"].endswith(
        os.path.join(d, "run_counter_collection.csv"))


def test_requires_passes_without_clock_only(tmp_path):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "roofline_pmc.py"), "path:x:1x1",
                        "--out", str(tmp_path / "r.json")], capture_output=True, text=True)
    assert p.returncode != 0 and "required" in p.stderr
