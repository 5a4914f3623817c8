# instruction mix of one kernel's ISA (development): kernel_isa.sh LIB symbol-substring
L=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$L/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin $1
$L/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --output=$T/g.co --targets=hipv4-amdgcn-amd-amdhsa--gfx950
$L/llvm-objdump -d --no-show-raw-insn $T/g.co > $T/g.s
python3 - "$T/g.s" "$2" <<'PY'
import sys, re, collections
txt = open(sys.argv[1]).read().split('\n')
pat = sys.argv[2]
cur = None; body = collections.defaultdict(list)
for ln in txt:
    m = re.match(r'^[0-9a-f]+ <(.*)>:', ln)
    if m: cur = m.group(1); continue
    if cur and ln.strip() and not ln.startswith('Disassembly'):
        body[cur].append(ln.strip().split()[0])
for k, v in body.items():
    if pat in k:
        c = collections.Counter()
        for op in v:
            c['v_' if op.startswith('v_') else 'ds_' if op.startswith('ds_') else 's_' if op.startswith('s_') else 'other'] += 1
        print(k[:90], len(v), dict(c))
PY
rm -rf $T
