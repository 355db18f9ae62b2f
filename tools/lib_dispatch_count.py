import csv,collections,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
step=0; lib=collections.Counter(); tot=collections.Counter()
for r in rows:
    n=r['Kernel_Name']
    if 'hyper_tick' in n: step+=1
    tot[step]+=1
    if 'at::native' in n or 'rocclr' in n or 'Cijk' in n or 'rocprim' in n or 'fillBuffer' in n: lib[(step,n[:100])]+=1
print("step index = number of optimizer hyper_tick kernels seen so far (step 0 = setup + first step)")
print("dispatches per step:", dict(tot))
print("library (at::native / rocclr / Cijk / rocprim / fillBuffer) dispatches by step:")
for k,v in sorted(lib.items()): print("  step %d: %4d x %s" % (k[0], v, k[1]))
