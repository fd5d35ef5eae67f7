"""Regenerate oracle/ipmc_oracle.c's orc_layout() from ip_mcmc_amd/_abi.py field lists."""
import importlib.util
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("abi", os.path.join(REPO, "ip_mcmc_amd", "_abi.py"))
abi = importlib.util.module_from_spec(spec)
spec.loader.exec_module(abi)
code = ("/* Struct layout as this C compiler sees include/ipmc.h (checked by tests/test_lib_exports.py). */\n"
        "#include <stddef.h>\nint orc_layout(int64_t* out) {\n  int i = 0;\n  out[i++] = (int64_t)sizeof(ipmc_model);\n")
for f, _ in abi.IpmcModel._fields_:
    code += f"  out[i++] = (int64_t)offsetof(ipmc_model, {f});\n"
code += "  out[i++] = (int64_t)sizeof(ipmc_sweep);\n"
for f, _ in abi.IpmcSweep._fields_:
    code += f"  out[i++] = (int64_t)offsetof(ipmc_sweep, {f});\n"
code += "  return i;\n}\n"
p = os.path.join(REPO, "oracle", "ipmc_oracle.c")
s = open(p).read()
a = s.index("/* Struct layout as this C compiler")
b = s.index("int orc_abi_version")
open(p, "w").write(s[:a] + code + "\n" + s[b:])
