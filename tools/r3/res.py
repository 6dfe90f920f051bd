"""Kernel resource usage from `make asm-ppo` / `make asm` remarks (stdin): name, VGPRs, AGPRs,
scratch, occupancy, VGPR / SGPR spills, LDS.  python tools/r3/res.py [name-regex] < remarks"""
import re, sys
pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": re.sub(r"_ZN12_GLOBAL__N_1\d+", "", m.group(1))}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
for r in rows:
    if pat and not pat.search(r["name"]):
        continue
    print(f'{r["name"][:48]:48s} v{r.get("VGPRs","?"):>4} a{r.get("AGPRs","?"):>3} scr{r.get("ScratchSize","?"):>4} '
          f'occ{r.get("Occupancy","?"):>2} vsp{r.get("VGPRs Spill","?"):>3} ssp{r.get("SGPRs Spill","?"):>3} lds{r.get("LDS Size","?"):>7}')
