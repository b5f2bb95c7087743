"""Build the package's native pieces in-tree: libmmfusion.so (hipcc, csrc/Makefile) and mmf_torch
(csrc/torch_bind.cpp: the eager module path's autograd nodes in C++ over libmmfusion.so's C-ABI,
compiled against the installed libtorch).  Used by __graft_entry__.build(); the built .so files
travel with the tree."""

from __future__ import annotations

import os
import subprocess
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")


def torch_ext_path() -> str:
    return os.path.join(HERE, "mmf_torch" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_torch_ext(force: bool = False) -> str:
    """g++ csrc/torch_bind.cpp -> mmf_torch<EXT_SUFFIX> next to this file (skipped when newer than
    its sources)."""
    import torch
    import torch.utils.cpp_extension as ce
    out = torch_ext_path()
    src = os.path.join(CSRC, "torch_bind.cpp")
    deps = [src, os.path.join(INCLUDE, "mmfusion.h"), __file__]
    if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    tlib = ce.library_paths()[0]
    tmp = f"{out}.{os.getpid()}.tmp"   # (concurrent builders -- pytest workers -- each write their own)
    abi = int(bool(torch._C._GLIBCXX_USE_CXX11_ABI))
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cmd = (["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-w", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
            "-DTORCH_EXTENSION_NAME=mmf_torch", "-DTORCH_API_INCLUDE_EXTENSION_H", "-D__HIP_PLATFORM_AMD__=1",
            "-DUSE_ROCM", f"-I{rocm}/include", f"-I{INCLUDE}", f"-I{sysconfig.get_paths()['include']}"]
           + [f"-I{p}" for p in ce.include_paths()]
           + [src, "-o", tmp, f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
              "-ltorch_python", f"-Wl,-rpath,{tlib}"])
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build_torch_ext(force=True))
