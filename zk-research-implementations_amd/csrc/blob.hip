// Proof blobs: canonical proof bytes, C ABI.
#include "host.hpp"

using namespace zkh;

extern "C" {

// ---- proof blobs ----
// Layout (include/zk_sumcheck.h "Proof blob"): "ZKSP", version 1, kind,
// field, 0, nrounds (u32 LE), claimed_sum (32 B), then per round m (u8) and
// m canonical 32-byte LE coefficients — for a GKR proof exactly the bytes the
// transcript absorbs in that round (fq_vec_to_bytes of the trimmed poly).
extern "C++" {
namespace {
constexpr uint8_t kBlobVersion = 1;

struct BlobWriter {
  uint8_t* out;
  size_t cap, len = 0;
  void put(const void* p, size_t n) {
    if (out && len + n <= cap) memcpy(out + len, p, n);
    len += n;
  }
  void u8(uint8_t v) { put(&v, 1); }
  void u32(uint32_t v) { put(&v, 4); }  // little-endian host
};

template <class F>
void blob_fe(BlobWriter& w, zk_repr repr, const zk_fe& x) {
  uint8_t b[32];
  canon_bytes<F>(in_mont<F>(repr, x), b);
  w.put(b, 32);
}

void blob_header(BlobWriter& w, int kind, zk_field field, uint32_t nrounds) {
  w.put("ZKSP", 4);
  w.u8(kBlobVersion);
  w.u8((uint8_t)kind);
  w.u8((uint8_t)field);
  w.u8(0);
  w.u32(nrounds);
}

struct BlobReader {
  const uint8_t* p;
  size_t len, off = 0;
  const uint8_t* take(size_t n) {
    require(off + n <= len, "proof blob truncated");
    const uint8_t* q = p + off;
    off += n;
    return q;
  }
};

// parse the header; returns kind
int blob_open(BlobReader& r, zk_field* field, uint32_t* nrounds) {
  const uint8_t* h = r.take(12);
  require(memcmp(h, "ZKSP", 4) == 0, "not a proof blob");
  require(h[4] == kBlobVersion, "unsupported proof blob version");
  require(h[5] == ZK_BLOB_GKR || h[5] == ZK_BLOB_SUMCHECK, "unknown proof blob kind");
  require(h[6] <= ZK_BLS12_381_FR && h[7] == 0, "bad proof blob header");
  *field = (zk_field)h[6];
  memcpy(nrounds, h + 8, 4);
  return h[5];
}

template <class F>
zk_fe blob_read_fe(BlobReader& r, zk_repr repr) {  // canonical bytes -> repr, rejects >= p
  zk_fe x;
  memcpy(x.limb, r.take(32), 32);
  const Fe c = from_zk(x);
  require(zk::fe_is_canonical<F>(c), "proof blob element >= modulus");
  return repr == ZK_REPR_MONTGOMERY ? to_zk(zk::fe_to_mont<F>(c)) : x;
}
}  // namespace
}  // extern "C++"

int zk_gkr_proof_to_blob(zk_field field, zk_repr repr, const zk_fe* coeffs, const uint8_t* ncoeffs, uint32_t nrounds,
                         const zk_fe* claimed_sum, uint8_t* out, size_t cap, size_t* out_len) {
  return guarded([&] {
    require(claimed_sum && out_len && (nrounds == 0 || (coeffs && ncoeffs)), "null argument");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      BlobWriter w{out, cap};
      blob_header(w, ZK_BLOB_GKR, field, nrounds);
      blob_fe<F>(w, repr, *claimed_sum);
      for (uint32_t k = 0; k < nrounds; ++k) {
        require(ncoeffs[k] <= 3, "round polynomial has more than 3 coefficients");
        w.u8(ncoeffs[k]);
        for (int i = 0; i < ncoeffs[k]; ++i) blob_fe<F>(w, repr, coeffs[3 * (size_t)k + i]);
      }
      *out_len = w.len;
      if (out) require(w.len <= cap, "output buffer too small");
    });
  });
}

int zk_sumcheck_proof_to_blob(zk_field field, zk_repr repr, const zk_fe* round_polys, uint32_t nrounds,
                              uint32_t poly_len, const zk_fe* claimed_sum, uint8_t* out, size_t cap, size_t* out_len) {
  return guarded([&] {
    require(claimed_sum && out_len && (nrounds == 0 || round_polys), "null argument");
    require(poly_len <= 255, "round polynomial too long for the blob format");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      BlobWriter w{out, cap};
      blob_header(w, ZK_BLOB_SUMCHECK, field, nrounds);
      blob_fe<F>(w, repr, *claimed_sum);
      for (uint32_t k = 0; k < nrounds; ++k) {
        w.u8((uint8_t)poly_len);
        for (uint32_t i = 0; i < poly_len; ++i) blob_fe<F>(w, repr, round_polys[(size_t)k * poly_len + i]);
      }
      *out_len = w.len;
      if (out) require(w.len <= cap, "output buffer too small");
    });
  });
}

int zk_proof_blob_info(const uint8_t* blob, size_t len, int* out_kind, zk_field* out_field, uint32_t* out_nrounds) {
  return guarded([&] {
    require(blob && out_kind && out_field && out_nrounds, "null argument");
    BlobReader r{blob, len};
    *out_kind = blob_open(r, out_field, out_nrounds);
  });
}

int zk_gkr_proof_from_blob(const uint8_t* blob, size_t len, zk_repr repr, zk_fe* out_coeffs, uint8_t* out_ncoeffs,
                           uint32_t cap_rounds, zk_fe* out_claimed_sum) {
  return guarded([&] {
    require(blob && out_claimed_sum, "null argument");
    BlobReader r{blob, len};
    zk_field field;
    uint32_t n;
    require(blob_open(r, &field, &n) == ZK_BLOB_GKR, "not a GKR sum-check proof blob");
    require(n <= cap_rounds && (n == 0 || (out_coeffs && out_ncoeffs)), "output buffer too small");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      *out_claimed_sum = blob_read_fe<F>(r, repr);
      for (uint32_t k = 0; k < n; ++k) {
        const uint8_t m = *r.take(1);
        require(m <= 3, "round polynomial has more than 3 coefficients");
        out_ncoeffs[k] = m;
        for (int i = 0; i < 3; ++i) out_coeffs[3 * (size_t)k + i] = i < m ? blob_read_fe<F>(r, repr) : zk_fe{};
      }
      require(r.off == len, "trailing bytes after the proof");
    });
  });
}

int zk_sumcheck_proof_from_blob(const uint8_t* blob, size_t len, zk_repr repr, zk_fe* out_round_polys,
                                size_t cap_elems, uint32_t* out_poly_len, zk_fe* out_claimed_sum) {
  return guarded([&] {
    require(blob && out_poly_len && out_claimed_sum, "null argument");
    BlobReader r{blob, len};
    zk_field field;
    uint32_t n;
    require(blob_open(r, &field, &n) == ZK_BLOB_SUMCHECK, "not a sum-check proof blob");
    dispatch(field, [&](auto f) {
      using F = decltype(f);
      *out_claimed_sum = blob_read_fe<F>(r, repr);
      uint32_t plen = 0;
      for (uint32_t k = 0; k < n; ++k) {
        const uint8_t m = *r.take(1);
        require(k == 0 || m == plen, "round polynomials of different lengths");
        plen = m;
        require((size_t)(k + 1) * m <= cap_elems && out_round_polys, "output buffer too small");
        for (uint32_t i = 0; i < m; ++i) out_round_polys[(size_t)k * m + i] = blob_read_fe<F>(r, repr);
      }
      *out_poly_len = plen;
      require(r.off == len, "trailing bytes after the proof");
    });
  });
}

int zk_gkr_verify_blob(const uint8_t* blob, size_t len, zk_transcript* transcript, int* out_verified,
                       zk_fe* out_final_claimed_sum, zk_fe* out_challenges, uint32_t cap_rounds) {
  int rc = ZK_OK;
  const int g = guarded([&] {
    require(blob && transcript && out_verified && out_final_claimed_sum, "null argument");
    BlobReader r{blob, len};
    zk_field field;
    uint32_t n;
    require(blob_open(r, &field, &n) == ZK_BLOB_GKR, "not a GKR sum-check proof blob");
    require(n <= cap_rounds && (n == 0 || out_challenges), "output buffer too small");
    std::vector<zk_fe> cf(3 * (size_t)std::max<uint32_t>(n, 1));
    std::vector<uint8_t> nc(std::max<uint32_t>(n, 1));
    zk_fe cs;
    if (zk_gkr_proof_from_blob(blob, len, ZK_REPR_CANONICAL, cf.data(), nc.data(), n, &cs) != ZK_OK)
      fail(ZK_EINVAL, g_last_error);
    zk_fe dummy;
    rc = zk_gkr_sumcheck_verify(field, ZK_REPR_CANONICAL, cf.data(), nc.data(), n, &cs, transcript, out_verified,
                                out_final_claimed_sum, n ? out_challenges : &dummy);
    if (rc != ZK_OK) fail(rc, g_last_error);
  });
  return g;
}

int zk_keccak256(const uint8_t* data, size_t len, uint8_t out[32]) {
  return guarded([&] {
    require(out && (data || len == 0), "null argument");
    zk::Keccak256 h;
    h.update(data, len);
    h.finalize_reset(out);
  });
}

}  // extern "C"
