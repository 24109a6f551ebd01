import csv,sys
f=sys.argv[1]
rows=sorted(csv.DictReader(open(f)),key=lambda r:int(r["Start_Timestamp"]))
# find sequences starting at k_preprocess
seqs=[];cur=None
for r in rows:
    n=r["Kernel_Name"]
    if "k_preprocess" in n:
        cur=[];seqs.append(cur)
    if cur is not None: cur.append(r)
import re
for s in seqs[-8:]:
    t0=int(s[0]["Start_Timestamp"])
    out=[]
    for r in s:
        n=r["Kernel_Name"]; n=re.sub(r"\(.*","",n).replace("void ","").replace("gs::","")
        d=(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1000
        out.append(f"{n[:18]}:{d:.1f}")
    print(" ".join(out))
