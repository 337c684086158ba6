"""Extract the reference's own known-answer data for the hot path into
tests/golden/reference_kats.json (inputs and expected outputs only).

Run in the authoring container (needs /root/reference); the JSON is committed
and is all the tests read. Each entry records the reference file:line it came
from. Values are canonical field elements (MontFp!("x") and Fq::from(x) both
denote the canonical integer x; negative Fq::from(-x) becomes p - x).
"""
import json
import re
import sys
from pathlib import Path

REF = Path("/root/reference/latticeum")
OUT = Path(__file__).resolve().parents[1] / "tests/golden/reference_kats.json"
P = (1 << 64) - (1 << 32) + 1
GL_NTT = REF / "crates/stark-rings/crates/ring/src/cyclotomic_ring/models/goldilocks/ntt.rs"
CHAL = REF / "crates/cyclotomic-rings/src/rings/goldilocks.rs"


def fn_body(src: str, name: str) -> str:
    i = src.index(f"fn {name}(")
    j = src.find("\n    #[test]", i)
    return src[i:j if j > 0 else len(src)]


def field_list(text: str):
    """Parse a Rust vec![...] of Fq::from(n) / Fq::zero() / Fq::one() / MontFp!("n")."""
    vals = []
    for m in re.finditer(r'MontFp!\("(\d+)"\)|Fq::from\((-?\d+)(?:u64)?\)|Fq::zero\(\)|Fq::one\(\)', text):
        if m.group(1) is not None:
            vals.append(int(m.group(1)) % P)
        elif m.group(2) is not None:
            vals.append(int(m.group(2)) % P)
        elif m.group(0) == "Fq::zero()":
            vals.append(0)
        else:
            vals.append(1)
    return vals


def line_of(path: Path, needle: str) -> int:
    for n, line in enumerate(path.read_text().splitlines(), 1):
        if needle in line:
            return n
    raise KeyError(needle)


def crt_kats():
    src = GL_NTT.read_text()
    out = {}
    for name in ("test_crt", "test_crt2"):
        body = fn_body(src, name)
        inp_txt, exp_txt = body.split("let expected")
        inp = field_list(inp_txt)
        inp += [0] * (24 - len(inp))  # test_poly.resize_with(D, Fq::zero)
        exp = field_list(exp_txt.split("serial_goldilock_crt_in_place")[0])
        assert len(inp) == 24 and len(exp) == 24, (name, len(inp), len(exp))
        out[name] = {
            "source": f"GL/ntt.rs:{line_of(GL_NTT, f'fn {name}(')}",
            "what": "serial_goldilock_crt_in_place then dehomogenize_fq3",
            "coeffs": inp, "crt_dehomogenized": exp,
        }
    for name in ("test_icrt", "test_icrt_2"):
        body = fn_body(src, name)
        exp_txt, ev_txt = body.split("let mut evaluations")
        exp = field_list(exp_txt)
        exp += [0] * (24 - len(exp))
        ev = field_list(ev_txt.split("homogenize_fq3")[0])
        assert len(exp) == 24 and len(ev) == 24
        out[name] = {
            "source": f"GL/ntt.rs:{line_of(GL_NTT, f'fn {name}(')}",
            "what": "homogenize_fq3 then serial_goldilock_icrt_in_place",
            "evaluations_dehomogenized": ev, "coeffs": exp,
        }
    return out


def challenge_kat():
    src = CHAL.read_text()
    body = src[src.index("fn test_small_challenge_from_random_bytes"):]
    bs = [int(x, 16) for x in re.findall(r"0x([0-9a-f]{2})", body.split("unwrap()")[0])]
    coeffs = [int(x) for x in re.findall(r"BigInt\(\[(\d+)\]\)", body)]
    assert len(bs) == 18 and len(coeffs) == 24
    return {"source": f"CR/rings/goldilocks.rs:{line_of(CHAL, 'fn test_small_challenge_from_random_bytes')}",
            "bytes": bs, "coeffs": coeffs}


def sage_vec(text: str, name: str):
    i = text.index(name)
    j = text.index("]", i)
    return [int(x) for x in re.findall(r"\b(\d{1,20})\b", text[text.index("[", i) + 1:j])]


def poseidon_kats():
    log = (REF / "session.log").read_text()
    v_i = log.index("v = vector(F, [")
    v = [int(x) for x in re.findall(r"\b(\d+)\b", log[v_i + 15:log.index("])", v_i)])]
    u_i = log.index("u = vector(F, [")
    u = [int(x) for x in re.findall(r"\b(\d+)\b", log[u_i + 15:log.index("])", u_i)])]
    assert len(v) == 16 and len(u) == 16
    init = (REF / "sages/initial_mds.sage").read_text()
    ext = (REF / "sages/external_initial_rounds.sage").read_text()
    inv = (REF / "sages/inverse_mds.sage").read_text()
    init_state = sage_vec(init, "initial_state")
    s = [int(x) for x in re.findall(r"F\((\d+)\)", ext[ext.index("s = ["):ext.index("consts_0")])]
    consts0 = [int(x) for x in re.findall(r"F\((\d+)\)", ext[ext.index("consts_0 = ["):])][:16]
    v2 = sage_vec(inv, "v = vector(")
    asm = sage_vec(inv, "after_sbox_mds = vector(")
    assert len(init_state) == 16 and len(s) == 16 and len(v2) == 16 and len(asm) == 16
    return {
        "P1_mds": {"source": "latticeum/session.log:62-120 (v*A with A = MDS16^T)",
                   "input": v, "mds16": u},
        "P2_initial_mds": {"source": "latticeum/sages/initial_mds.sage:4-23 + external_initial_rounds.sage:6-23",
                           "input": init_state, "mds16": s},
        "P3_round0": {"source": "latticeum/sages/inverse_mds.sage:29-76 (consts_0: external_initial_rounds.sage:25-42)",
                      "input": v2, "round0_consts": consts0,
                      "mds_sbox_mds": asm},
    }


ROT = REF / "crates/cyclotomic-rings/src/rotation.rs"


def rot_kat():
    """test_rot_lin_combination: v_0 = sum_i RotSum(rho_i, flatten(theta_i)) over Phi_72"""
    src = ROT.read_text()
    body = fn_body(src, "test_rot_lin_combination")
    rho_txt, rest = body.split("let theta_s")[0], body.split("let theta_s")[1]
    theta_txt, exp_txt = rest.split("let res")[0], rest.split("let expected")[1]
    rho, theta, exp = field_list(rho_txt), field_list(theta_txt), field_list(exp_txt)
    n = len(rho) // 24
    assert len(rho) == 24 * n and len(theta) == 72 * n and len(exp) == 72, (len(rho), len(theta), len(exp))
    return {"source": f"CR/rotation.rs:{line_of(ROT, 'fn test_rot_lin_combination(')}",
            "rho_coeff": [rho[24 * i:24 * i + 24] for i in range(n)],
            "theta_ntt": [theta[72 * i:72 * i + 72] for i in range(n)],
            "expected_ntt": exp}


def main() -> int:
    kats = {
        "_comment": "Known-answer data extracted from the reference's own tests/sage logs by "
                    "tools/gen_golden_kats.py. Canonical field elements (p = 2^64-2^32+1).",
        "crt": crt_kats(),
        "short_challenge": challenge_kat(),
        "ajtai_closed_form": {
            "source": "LF/commitment/commitment_scheme.rs:124-159",
            "kappa": 9, "n": 1 << 15, "witness_scalar": 2,
            "rule": "A[i][j] = scalar(i*n + j); cm[i] = scalar(n*(2*i*n + n - 1))"},
        "gadget": {
            "source": "SR/balanced_decomposition/mod.rs:469-515",
            "b": 2, "padding": 4,
            "input_scalars": [15, P - 15],
            "expected_digits": [[1, 1, 1, 1], [P - 1, P - 1, P - 1, P - 1]]},
        "get_fhat": {
            "source": "LF/arith.rs:455-502",
            "f_coeffs": [[1, 2, 3] + [0] * 21, [4, 5, 6] + [1] * 21],
            "expected_mle_first_ntt_slots": [[[1, 2, 3, 0, 0, 0, 0, 0], [4, 5, 6, 1, 1, 1, 1, 1]],
                                             [[0] * 8, [1] * 8], [[0] * 8, [1] * 8]]},
        "poseidon2": poseidon_kats(),
        "rot_lin_combination": rot_kat(),
    }
    OUT.parent.mkdir(parents=True, exist_ok=True)
    OUT.write_text(json.dumps(kats, indent=1))
    print("wrote", OUT)
    return 0


if __name__ == "__main__":
    sys.exit(main())
