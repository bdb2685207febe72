"""Per-kernel, per-grid-size duration summary of a rocprofv3 SQLite
database (``rocprofv3 --kernel-trace -d DIR -o NAME`` writes
DIR/.../NAME_results.db):

    python tools/rocpd_stats.py path/to/NAME_results.db [name-filter]
"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    flt = sys.argv[2] if len(sys.argv) > 2 else "pyas"
    cur = db.cursor()
    names = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    ks = next(n for n in names if n.startswith("rocpd_kernel_dispatch"))
    ss = next(n for n in names if n.startswith("rocpd_info_kernel_symbol"))
    q = (f"select s.kernel_name, k.grid_size_x / k.workgroup_size_x, count(*), avg(k.end - k.start), "
         f"min(k.end - k.start), max(k.end - k.start), s.arch_vgpr_count, s.group_segment_size "
         f"from {ks} k join {ss} s on k.kernel_id = s.id where s.kernel_name like ? "
         f"group by s.kernel_name, k.grid_size_x order by min(k.start)")
    print("kernel,workgroups,calls,avg_us,min_us,max_us,vgpr,lds")
    for name, wg, n, avg, mn, mx, vgpr, lds in cur.execute(q, (f"%{flt}%",)):
        print(f"{name},{wg},{n},{avg / 1e3:.1f},{mn / 1e3:.1f},{mx / 1e3:.1f},{vgpr},{lds}")


if __name__ == "__main__":
    main()
