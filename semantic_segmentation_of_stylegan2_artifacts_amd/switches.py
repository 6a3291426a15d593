"""The environment switches the product path reads: all of them, read once at import.

Each one is an A/B switch kept for a measured reason (DESIGN.md section 7 names the record); the
defaults are the measured winners.  Nothing else in the package or in ``csrc/`` reads the
environment (``tests/test_switches.py`` checks the sources), and ``bench.py`` prints every
non-default value -- and any unknown ``MSU_*`` variable, i.e. a stale switch that would be
silently ignored -- into its JSON line's ``config.switches``.
"""
import os
import warnings

# name -> (default, what it selects, A/B record)
SWITCHES = {
    "MSU_LIB_OVERRIDE": ("", "path of another libmsunet_hip.so (tools/build_exp.sh ablation builds)",
                         "DESIGN 4c"),
    "MSU_WGRAD_SIDE": ("1", "0: every weight gradient on the main stream (determinism bisection)",
                       "DESIGN 4b, 7 (side stream +1.6 %)"),
    "MSU_ATTN_QKV": ("1", "0: the unfused stage-0 qkv Linear + window attention + proj",
                     "DESIGN 4d (r04c: +0.8 %)"),
    "MSU_GEMM_ROUTE": ("", "force a GEMM route: lib (hipBLASLt) / tok / nt",
                       "DESIGN 7 (r03c: hand-written +2.7 % over hipBLASLt)"),
    "MSU_NT_PP": ("0", "1: the ping-pong NT GEMM (gemm_pp.h) where it tiles exactly, else the persistent one",
                  "DESIGN 7 (r05g: 0.72-0.98x of the persistent kernel; no-store ablation 1.07-1.66x)"),
    "MSU_LINBWD": ("1", "0: stage-0 Linear backward as input-gradient GEMM + side-stream weight gradient",
                   "DESIGN 7 (r03af: one-pass +1.4 %)"),
    "MSU_CONV_SIDE": ("1", "0: the refine-conv weight gradients on the main stream",
                      "DESIGN 7 (r04s: side +0.2 %)"),
    "MSU_TAIL": ("1", "0: LayerNorm parameter-gradient partials summed by a colsum launch, not in the kernel",
                 "DESIGN 7 (r05i: +0.5 %, host -4 ms/step)"),
    "MSU_ATTN_AUX": ("1", "0: each attention backward rebuilds its relative-bias image instead of reusing the "
                     "forward's workspace", "DESIGN 7 (r05az)"),
    "MSU_MLP_INFER": ("1", "0: no-grad stage-0 MLPs on the token-GEMM pair instead of the fused kernel",
                      "DESIGN 7 (r05am: +1.3 %)"),
    "MSU_MLP_LN": ("1", "0: no-grad stage-0 blocks run norm2's residual-add LayerNorm as its own kernel before the "
                   "fused MLP", "DESIGN 7 (r05at)"),
    "MSU_MLP_TRAIN": ("1", "0: training stage-0 MLPs on the token-GEMM pair (H and GELU(H) stored) instead of "
                      "the fused kernel storing H only", "DESIGN 7 (r05ao)"),
    "MSU_LN_DEFER": ("1", "0: each LayerNorm backward sums its parameter-gradient partials itself (in-kernel "
                     "tail) instead of one batched reduction per width", "DESIGN 7 (r06)"),
    "MSU_NT_DYN": ("0", "1: the NT GEMM's two-stage kernel claims tiles from a per-XCD device queue (measured "
                   "-0.3 % step, 1.8 % slower standalone: r06q/r06r)", "DESIGN 7 (r06)"),
    "MSU_CONV_DYN": ("1", "0: the refine-conv kernel's static tile schedule (blockIdx.x + k * gridDim.x) instead "
                     "of the device tile queue", "DESIGN 7 (r06)"),
    "MSU_CONV_WGRAD_BLOCKS": ("256", "persistent workgroups of the refine-conv weight gradient (one per CU by "
                              "default; fewer leave CUs to the main stream)", "DESIGN 7 (r04ac, r06)"),
    "MSU_MLP_S1": ("1", "0: the stage-1 training MLPs on the GEMM pair (H and GELU(H) stored) instead of the "
                   "fused kernel streaming its weights through an LDS ring", "DESIGN 7 (r06)"),
    "MSU_RES_HANDOFF": ("1", "0: a stage's first Swin block sums its input's two gradients (norm1 LayerNorm, norm2 "
                        "residual) with an ATen add instead of inside the LayerNorm backward", "DESIGN 7 (r06)"),
    "MSU_GRAPH": ("auto", "HIP-graph replay of the step: 1 / 0 / auto (replay when launch-bound)",
                  "DESIGN 4b (512^2: 401 vs 249-307 img/s)"),
    "MSU_GRAPH_SIDE": ("0", "1: fork the side stream into the captured graph (nondeterministic on ROCm 7.2)",
                       "DESIGN 4b (r03h)"),
}

VALUES = {name: os.environ.get(name, d[0]) for name, d in SWITCHES.items()}


def get(name):
    """The value of a registered switch (a KeyError for an unregistered name)."""
    return VALUES[name]


def on(name):
    """A registered 0 / 1 switch as a bool."""
    return VALUES[name] != "0"


def unknown():
    """``MSU_*`` environment variables this package does not read (stale or misspelt switches)."""
    return sorted(k for k in os.environ if k.startswith("MSU_") and k not in SWITCHES)


def report():
    """{name: value} of every switch set away from its default, plus unknown ``MSU_*`` ones."""
    out = {k: v for k, v in VALUES.items() if v != SWITCHES[k][0]}
    out.update({k: os.environ[k] + " (unknown: ignored)" for k in unknown()})
    return out


if unknown():
    warnings.warn(f"environment variables not read by this package (ignored): {', '.join(unknown())}")
