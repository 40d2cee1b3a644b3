import sqlite3, sys, glob
for db in sys.argv[1:]:
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    kd = [t for t in tabs if 'kernel_dispatch' in t.lower() or t.lower()=='kernels']
    print("==", db)
    # try the 'kernels' view
    t = 'kernels' if 'kernels' in tabs else kd[0]
    cols = [r[1] for r in c.execute(f"pragma table_info({t})")]
    nm = 'name' if 'name' in cols else ('kernel_name' if 'kernel_name' in cols else None)
    q = f"select {nm}, count(*), avg(end-start)/1e6, min(end-start)/1e6 from {t} group by {nm} order by sum(end-start) desc limit 8"
    for r in c.execute(q):
        print(f"  {r[0][:70]:70s} n={r[1]:4d} avg={r[2]:.4f} ms min={r[3]:.4f}")
