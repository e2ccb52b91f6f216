import sqlite3, sys
c = sqlite3.connect(sys.argv[1]); cur = c.cursor()
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 4
rows = cur.execute("select name, count(*), sum(end-start), avg(end-start) from kernels group by name order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"total kernel ms/step {tot/1e6/steps:.2f}  launches/step {sum(r[1] for r in rows)/steps:.0f}")
for n,cnt,s,a in rows[:int(sys.argv[3]) if len(sys.argv)>3 else 30]:
    short = n.replace('(anonymous namespace)::','').split('(')[0][:90]
    print(f"{s/1e6/steps:8.2f} ms {100*s/tot:5.1f}% n={cnt/steps:6.1f} avg={a/1e3:8.1f}us  {short}")
