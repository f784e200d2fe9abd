#!/usr/bin/env python3
"""Extract golden vectors for the ESP bulk-crypto path from the reference tree.

Run HERE (the survey/build container), never on the GPU box: it reads
/root/reference as text.  It parses the C initialisers of DPDK's own
known-answer tests (vendored in the reference at dpdk/app/test/) and writes
plain-data JSON fixtures next to this script:

  esp_packets.json   complete ESP tunnel packets (outer IP | ESP | IV | CT | ICV)
                     test_cryptodev_security_ipsec_test_vectors.h:22,127,226,540,2047
  gcm_aead.json      AES-GCM AEAD KATs (128/192/256-bit keys, AAD, empty PT)
                     test_cryptodev_aead_test_vectors.h:88-434,1037-1687,1740-1793
  cbc_hmac_sha1.json AES-CBC + HMAC-SHA1 chained KATs (encrypt-then-MAC over CT)
                     test_cryptodev_aes_test_vectors.h:1492,2187,2309
  eta_esp_packets.json  complete ESP tunnel packets, AES-CBC + HMAC-SHA2-256/384/512
                     test_cryptodev_security_ipsec_test_vectors.h:744,1721
  ctr_hmac_sha1.json AES-CTR (full 128-bit counter) + HMAC-SHA1 chained KATs
                     test_cryptodev_aes_test_vectors.h:1221,1311,1358,1447

The JSON holds only inputs and expected outputs (hex strings); no reference
source text is stored.  Usage:  python tests/golden/make_golden.py
"""
import json
import os
import re
import sys

REF = os.environ.get("FSTACK_REF", "/root/reference")
TESTDIR = os.path.join(REF, "dpdk", "app", "test")
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# A small parser for C designated initialisers: { .a = { .b = 1, ... }, ... }

def strip_comments(src):
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def find_block(src, pos):
    """src[pos] == '{' -> index one past the matching '}'."""
    depth = 0
    for i in range(pos, len(src)):
        if src[i] == "{":
            depth += 1
        elif src[i] == "}":
            depth -= 1
            if depth == 0:
                return i + 1
    raise ValueError("unbalanced braces")


def split_top(body):
    """Split 'a, b, {c, d}, e' at top-level commas."""
    parts, depth, cur = [], 0, []
    for ch in body:
        if ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    tail = "".join(cur).strip()
    if tail:
        parts.append(tail)
    return parts


def parse_value(v):
    v = v.strip()
    if v.startswith("{"):
        inner = v[1:find_block(v, 0) - 1]
        items = split_top(inner)
        if items and all(it.startswith(".") for it in items):
            out = {}
            for it in items:
                k, _, val = it.partition("=")
                keys = k.strip()[1:].split(".")
                d = out
                for kk in keys[:-1]:
                    d = d.setdefault(kk, {})
                d[keys[-1]] = parse_value(val)
            return out
        return [parse_value(it) for it in items]
    try:
        return int(v, 0)
    except ValueError:
        return v


def parse_structs(path, type_re):
    src = strip_comments(open(path).read())
    out = {}
    for m in re.finditer(type_re + r"\s+(\w+)\s*=\s*\{", src):
        start = m.end() - 1
        end = find_block(src, start)
        out[m.group(1)] = parse_value(src[start:end])
    return out


def parse_defines(path):
    src = strip_comments(open(path).read())
    out = {}
    for m in re.finditer(r"#define\s+(\w+)\s+(0x[0-9a-fA-F]+|\d+)\s*$", src, flags=re.M):
        out[m.group(1)] = int(m.group(2), 0)
    return out


def parse_arrays(path):
    """uint8_t arrays; a declared size pads the initialiser with zeros (C rule)."""
    src = strip_comments(open(path).read())
    defs = parse_defines(path)
    out = {}
    for m in re.finditer(r"static\s+(?:const\s+)?uint8_t\s+(\w+)\s*\[\s*(\w*)\s*\]\s*=\s*\{", src):
        start = m.end() - 1
        end = find_block(src, start)
        body = src[start + 1:end - 1].strip()
        if body.startswith('"'):
            # brace-enclosed string literal(s): C concatenates them, plus NUL
            text = "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', body))
            vals = list(text.encode("latin-1").decode("unicode_escape").encode("latin-1")) + [0]
        else:
            vals = [x for x in parse_value(src[start:end]) if isinstance(x, int)]
        size = m.group(2)
        if size:
            n = int(size, 0) if size[0].isdigit() else defs[size]
            vals = vals + [0] * (n - len(vals))
        out[m.group(1)] = vals
    out["__defines__"] = defs
    return out


def hexs(b):
    return bytes(b).hex()


def data_of(field, arrays, n=None):
    d = field["data"]
    if isinstance(d, str):
        d = arrays[d]
    d = [x for x in d if isinstance(x, int)]
    if n is None:
        n = field.get("len", len(d))
    if isinstance(n, str):
        n = arrays["__defines__"][n]
    assert len(d) >= n, "initialiser shorter than .len"
    return d[:n]


# --------------------------------------------------------------------------

def esp_packets():
    path = os.path.join(TESTDIR, "test_cryptodev_security_ipsec_test_vectors.h")
    structs = parse_structs(path, r"struct\s+ipsec_test_data")
    names = ["pkt_aes_128_gcm", "pkt_aes_192_gcm", "pkt_aes_256_gcm",
             "pkt_aes_256_gcm_v6", "pkt_aes_128_gcm_frag"]
    out = []
    for name in names:
        s = structs[name]
        aead = s["xform"]["aead"]["aead"]
        klen = aead["key"]["length"]
        key = data_of(s["key"], {}, klen)
        salt = data_of(s["salt"], {})
        outer = s["output_text"]["data"][: s["output_text"]["len"]]
        inner = s["input_text"]["data"][: s["input_text"]["len"]]
        ver = outer[0] >> 4
        iphl = (outer[0] & 0xF) * 4 if ver == 4 else 40
        esp = outer[iphl:]
        xf = s["ipsec_xform"]
        out.append({
            "name": name,
            "source": "dpdk/app/test/test_cryptodev_security_ipsec_test_vectors.h",
            "mode": "gcm",
            "key": hexs(key),
            "salt": hexs(salt),
            "spi": xf["spi"],
            "esn": int(xf.get("options", {}).get("esn", 0)),
            "esn_hi": int(xf.get("esn", {}).get("hi", 0)) if isinstance(xf.get("esn"), dict) else 0,
            "digest_len": aead["digest_length"],
            "outer_hdr_len": iphl,
            "esp_record": hexs(esp),
            "inner_packet": hexs(inner),
        })
    return out


def gcm_aead():
    path = os.path.join(TESTDIR, "test_cryptodev_aead_test_vectors.h")
    arrays = parse_arrays(path)
    structs = parse_structs(path, r"static\s+const\s+struct\s+aead_test_data")
    out = []
    for name, s in structs.items():
        if s.get("algo") != "RTE_CRYPTO_AEAD_AES_GCM":
            continue
        if "SGL" in name:
            continue
        iv = data_of(s["iv"], arrays)
        if len(iv) != 12:           # opencrypto GCM requires a 12-byte IV (cryptosoft.c:1093)
            continue
        aad = data_of(s["aad"], arrays)
        extra = {}
        if len(aad) > 32 and s["aad"]["data"] == "gcm_aad_text":
            # test_cryptodev.c:8969-8973 fills a large AAD by repeating its
            # first 32 bytes before running the case; store that rule.
            extra = {"aad_fill": "repeat32", "aad_len": len(aad)}
            aad = aad[:32]
        pt = data_of(s["plaintext"], arrays)
        ct = data_of(s["ciphertext"], arrays)
        tag = data_of(s["auth_tag"], arrays)
        out.append({
            "name": name,
            "source": "dpdk/app/test/test_cryptodev_aead_test_vectors.h",
            "key": hexs(data_of(s["key"], arrays)),
            "iv": hexs(iv), "aad": hexs(aad), "plaintext": hexs(pt),
            "ciphertext": hexs(ct), "tag": hexs(tag), **extra,
        })
    return out


def cbc_hmac_sha1():
    path = os.path.join(TESTDIR, "test_cryptodev_aes_test_vectors.h")
    arrays = parse_arrays(path)
    structs = parse_structs(path, r"static\s+const\s+struct\s+blockcipher_test_data")
    out = []
    for name in ["aes_test_data_4", "aes_test_data_13", "aes_test_data_11"]:
        s = structs[name]
        e = {
            "name": name,
            "source": "dpdk/app/test/test_cryptodev_aes_test_vectors.h",
            "cipher_key": hexs(data_of(s["cipher_key"], arrays)),
            "iv": hexs(data_of(s["iv"], arrays)),
            "plaintext": hexs(data_of(s["plaintext"], arrays)),
            "ciphertext": hexs(data_of(s["ciphertext"], arrays)),
        }
        if s.get("auth_algo") == "RTE_CRYPTO_AUTH_SHA1_HMAC":
            e["auth_key"] = hexs(data_of(s["auth_key"], arrays))
            e["digest"] = hexs(data_of(s["digest"], arrays))
            e["truncated_len"] = s["digest"].get("truncated_len", 20)
        out.append(e)
    return out


def eta_esp_packets():
    """ESP packets of CBC + HMAC-SHA2-256/384/512 SAs (ICV = half the hash,
    RFC 4868: 16, 24, 32 bytes)."""
    path = os.path.join(TESTDIR, "test_cryptodev_security_ipsec_test_vectors.h")
    structs = parse_structs(path, r"struct\s+ipsec_test_data")
    modes = {"RTE_CRYPTO_AUTH_SHA256_HMAC": "cbc-hmac-sha256", "RTE_CRYPTO_AUTH_SHA384_HMAC": "cbc-hmac-sha384",
             "RTE_CRYPTO_AUTH_SHA512_HMAC": "cbc-hmac-sha512"}
    out = []
    for name in ["pkt_aes_128_cbc_hmac_sha256", "pkt_aes_128_cbc_hmac_sha256_v6",
                 "pkt_aes_128_cbc_hmac_sha384", "pkt_aes_128_cbc_hmac_sha512"]:
        s = structs[name]
        ch = s["xform"]["chain"]
        cipher, auth = ch["cipher"]["cipher"], ch["auth"]["auth"]
        assert cipher["algo"] == "RTE_CRYPTO_CIPHER_AES_CBC" and auth["algo"] in modes
        outer = s["output_text"]["data"][: s["output_text"]["len"]]
        inner = s["input_text"]["data"][: s["input_text"]["len"]]
        ver = outer[0] >> 4
        iphl = (outer[0] & 0xF) * 4 if ver == 4 else 40
        out.append({
            "name": name,
            "source": "dpdk/app/test/test_cryptodev_security_ipsec_test_vectors.h",
            "mode": modes[auth["algo"]],
            "cipher_key": hexs(data_of(s["key"], {}, cipher["key"]["length"])),
            "auth_key": hexs(data_of(s["auth_key"], {}, auth["key"]["length"])),
            "digest_len": auth["digest_length"],
            "spi": s["ipsec_xform"]["spi"],
            "outer_hdr_len": iphl,
            "esp_record": hexs(outer[iphl:]),
            "inner_packet": hexs(inner),
        })
    return out


def cipher_esp_packets():
    """ESP packets of cipher-only SAs (esp_init's CSP_MODE_CIPHER: an
    encryption algorithm and no authentication, xform_esp.c:230-231):
    pkt_aes_128_cbc_null is AES-128-CBC with RTE_CRYPTO_AUTH_NULL, an ingress
    vector, so the ESP packet is its input and the inner packet its output."""
    path = os.path.join(TESTDIR, "test_cryptodev_security_ipsec_test_vectors.h")
    structs = parse_structs(path, r"struct\s+ipsec_test_data")
    out = []
    for name in ["pkt_aes_128_cbc_null"]:
        s = structs[name]
        ch = s["xform"]["chain"]
        cipher, auth = ch["cipher"]["cipher"], ch["auth"]["auth"]
        assert cipher["algo"] == "RTE_CRYPTO_CIPHER_AES_CBC" and auth["algo"] == "RTE_CRYPTO_AUTH_NULL"
        assert s["ipsec_xform"]["direction"] == "RTE_SECURITY_IPSEC_SA_DIR_INGRESS"
        esp_pkt = s["input_text"]["data"][: s["input_text"]["len"]]
        inner = s["output_text"]["data"][: s["output_text"]["len"]]
        iphl = (esp_pkt[0] & 0xF) * 4
        out.append({
            "name": name,
            "source": "dpdk/app/test/test_cryptodev_security_ipsec_test_vectors.h",
            "mode": "cbc-null",
            "cipher_key": hexs(data_of(s["key"], {}, cipher["key"]["length"])),
            "iv": hexs(data_of(s["iv"], {}, cipher["iv"]["length"])),
            "spi": s["ipsec_xform"]["spi"],
            "outer_hdr_len": iphl,
            "esp_record": hexs(esp_pkt[iphl:]),
            "inner_packet": hexs(inner),
        })
    return out


def ctr_hmac_sha1():
    """AES-CTR chained with HMAC-SHA1 (digest over the ciphertext); the IV is
    the whole initial counter block (16 bytes) or a 12-byte nonce whose
    32-bit counter starts at 1 (RFC 3686 layout, test_cryptodev_blockcipher.c)."""
    path = os.path.join(TESTDIR, "test_cryptodev_aes_test_vectors.h")
    arrays = parse_arrays(path)
    structs = parse_structs(path, r"static\s+const\s+struct\s+blockcipher_test_data")
    out = []
    for name in ["aes_test_data_1", "aes_test_data_3", "aes_test_data_1_IV_12_bytes",
                 "aes_test_data_3_IV_12_bytes"]:
        s = structs[name]
        assert s["crypto_algo"] == "RTE_CRYPTO_CIPHER_AES_CTR" and s["auth_algo"] == "RTE_CRYPTO_AUTH_SHA1_HMAC"
        out.append({
            "name": name,
            "source": "dpdk/app/test/test_cryptodev_aes_test_vectors.h",
            "cipher_key": hexs(data_of(s["cipher_key"], arrays)),
            "iv": hexs(data_of(s["iv"], arrays)),
            "plaintext": hexs(data_of(s["plaintext"], arrays)),
            "ciphertext": hexs(data_of(s["ciphertext"], arrays)),
            "auth_key": hexs(data_of(s["auth_key"], arrays)),
            "digest": hexs(data_of(s["digest"], arrays)),
            "truncated_len": s["digest"].get("truncated_len", 20),
        })
    return out


def main():
    if not os.path.isdir(TESTDIR):
        print("reference tree not found at %s" % TESTDIR, file=sys.stderr)
        return 1
    for fname, fn in (("esp_packets.json", esp_packets), ("gcm_aead.json", gcm_aead),
                      ("cbc_hmac_sha1.json", cbc_hmac_sha1), ("eta_esp_packets.json", eta_esp_packets),
                      ("ctr_hmac_sha1.json", ctr_hmac_sha1), ("cipher_esp_packets.json", cipher_esp_packets)):
        vecs = fn()
        with open(os.path.join(OUT, fname), "w") as f:
            json.dump(vecs, f, indent=1)
        print("%s: %d vectors" % (fname, len(vecs)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
