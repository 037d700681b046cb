// pir_serve.cpp -- the PIR server process of the reference (src/server/server.go), natively over
// the MI355X engine: TLS stream (src/common/network.go:125-162), one request-type byte then a
// msgpack request; the answer is msgpack(error) then msgpack(response) (server.go:53-125).
//
//   SETUP_REQUEST (0)        SetupRequest  -> SetupResponse   (server.go:295-331: setSystemParams,
//                            synthetic database of client.cpp:16-33, encode across files --
//                            here computed on the GPU by pir_engine_encode_across_dev)
//   TREE_SEARCH_REQUEST (1)  TreeSearchRequest{Key} -> TreeSearchResponse{Results, PartyIndex,
//                            ServerLatency, ReceiveTime, SendTime}   (tree.go:17-101)
//   MULTIPARTY_SEARCH_REQUEST (3)  MultipartySearchRequest{Key} -> MultipartySearchResponse{
//                            Results, ServerLatency, ReceiveTime, SendTime}  (multiparty.go:16-103,
//                            Mode 1: shares of the sqrt(N) DPF key scanned on the GPU)
//   HOLLANTI_SEARCH_REQUEST (4)    HollantiSearchRequest{Key [][]byte} -> HollantiSearchResponse{
//                            Results, ServerLatency, ReceiveTime, SendTime}  (hollanti.go:16-112,
//                            Mode 3: explicit coefficient vectors scanned on the GPU; the shard
//                            encoded within files, client.cpp:99-103, on the host)
//   CD732_SEARCH_REQUEST (5)  CD732SearchRequest{Key} -> CD732SearchResponse{Results,
//                            ServerLatency, ReceiveTime, SendTime}  (cd732.go:16-100, Mode 4: the
//                            covering-design key's NUM_CD_KEYS shares scanned on the GPU; the
//                            reference's handler also frees the server after every query,
//                            cd732.go:96 -- not inherited)
//   TEST_REQUEST (7)         TestRequest{Msg} -> TestResponse{Msg}
// Structs travel as msgpack maps keyed by the Go field names (the go-msgpack MsgpackHandle
// default).  Durations are int64 nanoseconds; times are msgpack timestamp extensions (-1).
// Byte strings are sent as bin and accepted as bin or str.  The exact byte form the Go client's
// un-vendored github.com/hashicorp/go-msgpack writes is not available here:
// parity at this boundary is unpinned beyond the struct shapes of src/common/common.go:51-81.
//
//   pir_serve --port 9000 --party 1 [--cert c.pem --key k.pem] [--device 0] [--byzantine 0]
//             [--max-conns N]      (exit after N connections; default: serve forever)
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/pir_engine.h"
#include "../../include/pir_server.h"

namespace {

enum : uint8_t {  // common.go:147-154
  SETUP_REQUEST = 0, TREE_SEARCH_REQUEST = 1, MULTIPARTY_SEARCH_REQUEST = 3,
  HOLLANTI_SEARCH_REQUEST = 4, CD732_SEARCH_REQUEST = 5, TEST_REQUEST = 7
};

// ---- msgpack (the subset the protocol uses) ----------------------------------------------
struct MVal {
  enum Kind { NIL, BOOL, INT, STR, BIN, ARR, MAP, EXT } kind = NIL;
  int64_t i = 0;  // BOOL / INT (uint64 above INT64_MAX is rejected)
  std::string s;  // STR / BIN / EXT payload
  std::vector<MVal> a;                        // ARR
  std::vector<std::pair<MVal, MVal>> m;       // MAP
  const MVal* get(const char* key) const {
    for (auto& kv : m)
      if ((kv.first.kind == STR || kv.first.kind == BIN) && kv.first.s == key) return &kv.second;
    return nullptr;
  }
  int64_t get_int(const char* key, int64_t dflt = 0) const {
    const MVal* v = get(key);
    return v && (v->kind == INT || v->kind == BOOL) ? v->i : dflt;
  }
};

struct Writer {
  std::string b;
  void u8(uint8_t v) { b.push_back((char)v); }
  void be(uint64_t v, int n) {
    for (int k = n - 1; k >= 0; --k) u8((uint8_t)(v >> (8 * k)));
  }
  void nil() { u8(0xc0); }
  void integer(int64_t v) {
    if (v >= 0 && v < 128) u8((uint8_t)v);
    else if (v < 0 && v >= -32) u8((uint8_t)(0xe0 | (v + 32)));
    else if (v >= 0) { u8(0xcf); be((uint64_t)v, 8); }
    else { u8(0xd3); be((uint64_t)v, 8); }
  }
  void str(const std::string& s) {
    const size_t n = s.size();
    if (n < 32) u8((uint8_t)(0xa0 | n));
    else if (n < 256) { u8(0xd9); be(n, 1); }
    else if (n < 65536) { u8(0xda); be(n, 2); }
    else { u8(0xdb); be(n, 4); }
    b += s;
  }
  void bin(const void* p, size_t n) {
    if (n < 256) { u8(0xc4); be(n, 1); }
    else if (n < 65536) { u8(0xc5); be(n, 2); }
    else { u8(0xc6); be(n, 4); }
    b.append((const char*)p, n);
  }
  void array(size_t n) {
    if (n < 16) u8((uint8_t)(0x90 | n));
    else if (n < 65536) { u8(0xdc); be(n, 2); }
    else { u8(0xdd); be(n, 4); }
  }
  void map(size_t n) {
    if (n < 16) u8((uint8_t)(0x80 | n));
    else if (n < 65536) { u8(0xde); be(n, 2); }
    else { u8(0xdf); be(n, 4); }
  }
  void timestamp(std::chrono::system_clock::time_point t) {  // ext -1, 96-bit form
    const auto ns = std::chrono::duration_cast<std::chrono::nanoseconds>(t.time_since_epoch()).count();
    const int64_t sec = ns / 1000000000, nsec = ns % 1000000000;
    u8(0xc7); u8(12); u8(0xff);
    be((uint64_t)nsec, 4);
    be((uint64_t)sec, 8);
  }
};

// a buffered reader over the TLS connection
struct Stream {
  SSL* ssl;
  uint8_t buf[1 << 16];
  int len = 0, pos = 0;
  bool fill() {  // false on EOF / error
    int r = SSL_read(ssl, buf, sizeof buf);
    if (r <= 0) return false;
    len = r;
    pos = 0;
    return true;
  }
  bool byte(uint8_t& v) {
    if (pos == len && !fill()) return false;
    v = buf[pos++];
    return true;
  }
  void need(uint8_t& v) {
    if (!byte(v)) throw std::runtime_error("connection closed inside a message");
  }
  uint64_t be(int n) {
    uint64_t v = 0;
    for (int k = 0; k < n; ++k) {
      uint8_t c;
      need(c);
      v = (v << 8) | c;
    }
    return v;
  }
  std::string bytes(uint64_t n) {
    if (n > (1ull << 30)) throw std::runtime_error("message field too large");
    std::string s;
    s.reserve(n);
    while (s.size() < n) {
      if (pos == len && !fill()) throw std::runtime_error("connection closed inside a message");
      const size_t take = std::min<size_t>(n - s.size(), (size_t)(len - pos));
      s.append((const char*)buf + pos, take);
      pos += (int)take;
    }
    return s;
  }
  MVal value(int depth = 0) {
    if (depth > 32) throw std::runtime_error("msgpack nesting too deep");
    uint8_t t;
    need(t);
    MVal v;
    auto arr = [&](uint64_t n) {
      v.kind = MVal::ARR;
      for (uint64_t k = 0; k < n; ++k) v.a.push_back(value(depth + 1));
    };
    auto mp = [&](uint64_t n) {
      v.kind = MVal::MAP;
      for (uint64_t k = 0; k < n; ++k) {
        MVal key = value(depth + 1);
        MVal val = value(depth + 1);
        v.m.emplace_back(std::move(key), std::move(val));
      }
    };
    auto sint = [&](int n) {
      const uint64_t u = be(n);
      const int sh = 64 - 8 * n;
      v.kind = MVal::INT;
      v.i = (int64_t)(u << sh) >> sh;
    };
    auto uint = [&](int n) {
      const uint64_t u = be(n);
      if (u > (uint64_t)INT64_MAX) throw std::runtime_error("integer out of range");
      v.kind = MVal::INT;
      v.i = (int64_t)u;
    };
    if (t <= 0x7f) { v.kind = MVal::INT; v.i = t; }
    else if (t >= 0xe0) { v.kind = MVal::INT; v.i = (int8_t)t; }
    else if ((t & 0xf0) == 0x80) mp(t & 0x0f);
    else if ((t & 0xf0) == 0x90) arr(t & 0x0f);
    else if ((t & 0xe0) == 0xa0) { v.kind = MVal::STR; v.s = bytes(t & 0x1f); }
    else switch (t) {
      case 0xc0: break;
      case 0xc2: v.kind = MVal::BOOL; v.i = 0; break;
      case 0xc3: v.kind = MVal::BOOL; v.i = 1; break;
      case 0xc4: v.kind = MVal::BIN; v.s = bytes(be(1)); break;
      case 0xc5: v.kind = MVal::BIN; v.s = bytes(be(2)); break;
      case 0xc6: v.kind = MVal::BIN; v.s = bytes(be(4)); break;
      case 0xc7: { const uint64_t n = be(1); (void)be(1); v.kind = MVal::EXT; v.s = bytes(n); break; }
      case 0xc8: { const uint64_t n = be(2); (void)be(1); v.kind = MVal::EXT; v.s = bytes(n); break; }
      case 0xc9: { const uint64_t n = be(4); (void)be(1); v.kind = MVal::EXT; v.s = bytes(n); break; }
      case 0xcc: uint(1); break;
      case 0xcd: uint(2); break;
      case 0xce: uint(4); break;
      case 0xcf: uint(8); break;
      case 0xd0: sint(1); break;
      case 0xd1: sint(2); break;
      case 0xd2: sint(4); break;
      case 0xd3: sint(8); break;
      case 0xd4: (void)be(1); v.kind = MVal::EXT; v.s = bytes(1); break;
      case 0xd5: (void)be(1); v.kind = MVal::EXT; v.s = bytes(2); break;
      case 0xd6: (void)be(1); v.kind = MVal::EXT; v.s = bytes(4); break;
      case 0xd7: (void)be(1); v.kind = MVal::EXT; v.s = bytes(8); break;
      case 0xd8: (void)be(1); v.kind = MVal::EXT; v.s = bytes(16); break;
      case 0xd9: v.kind = MVal::STR; v.s = bytes(be(1)); break;
      case 0xda: v.kind = MVal::STR; v.s = bytes(be(2)); break;
      case 0xdb: v.kind = MVal::STR; v.s = bytes(be(4)); break;
      case 0xdc: arr(be(2)); break;
      case 0xdd: arr(be(4)); break;
      case 0xde: mp(be(2)); break;
      case 0xdf: mp(be(4)); break;
      default: throw std::runtime_error("unsupported msgpack type");
    }
    return v;
  }
};

bool send_all(SSL* ssl, const std::string& b) {
  size_t off = 0;
  while (off < b.size()) {
    const int w = SSL_write(ssl, b.data() + off, (int)std::min<size_t>(b.size() - off, 1 << 20));
    if (w <= 0) return false;
    off += (size_t)w;
  }
  return true;
}

// ---- the server (one party, one engine) ---------------------------------------------------
struct Server {
  int party = 1, device = 0, byzantine = 0;
  std::mutex mu;
  pir_engine_t* eng = nullptr;
  // of the current engine (the params globals may move on): mode, answer rows, record bytes,
  // tree key length, multiparty (p, t), NUM_CD_KEYS_NEEDED, Hollanti coefficient-vector length
  int mode = -1, nq = 0, efs = 0, key_len = 0, p = 0, t = 0, cd_needed = 0;
  uint64_t num_files = 0;
};
Server g;

std::string setup(const MVal& req) {  // server.go:295-331
  const int log_files = (int)req.get_int("LogNumFiles"), fsz = (int)req.get_int("FileSizeBytes");
  const int t = (int)req.get_int("T", 1), k = (int)req.get_int("K", 1), r = (int)req.get_int("R");
  const int b = (int)req.get_int("B"), rho = (int)req.get_int("Rho", 1);
  const int mode = (int)req.get_int("Mode"), mac = (int)req.get_int("CheckMAC");
  if (mode != 0 && mode != 1 && mode != 3 && mode != 4)
    return "only the tree (0), multiparty (1), Hollanti (3) and covering-design (4) modes are "
           "served by this engine";
  if (mac != 0) return "CheckMAC setups are outside this engine's scope";
  if (mode == 0 && (t != 1 || b != 0)) return "tree mode needs T = 1 and B = 0";
  if (mode == 1 && t < 1) return "multiparty mode needs T >= 1";
  if (log_files < 0 || log_files > 40 || fsz < 1 || k < 1 || k > 16 || r < 0 || rho < 1 || b < 0)
    return "bad setup parameters";
  // the process-global sizing (params.cpp) and the engine change together, under g.mu: a
  // concurrent TREE_SEARCH sees either the old engine and its sizes or the new ones
  std::lock_guard<std::mutex> lk(g.mu);
  if (g.eng) pir_engine_destroy(g.eng);
  g.eng = nullptr;
  g.key_len = 0;
  g.mode = -1;
  setSystemParams(log_files, fsz, t, k, r, b, rho, mac, mode);
  if (g.party > NUM_PARTIES) return "this server's party index exceeds NUM_PARTIES";
  const int rounds = mode == 1 ? NUM_RSS_KEYS : (mode == 4 ? NUM_CD_KEYS : NUM_ROUNDS);
  if (rounds < 1 || rounds > PIR_MAX_ROUNDS)
    return "answer rows outside [1,16] (NUM_ROUNDS / NUM_RSS_KEYS / NUM_CD_KEYS)";
  pir_engine_config c{};
  c.device = g.device;
  // the party count only sizes tree-DPF keys (modes 1, 3 and 4 answer other key forms); the
  // party index also selects the encode-across evaluation point gf_pow(party, j) (client.cpp:
  // 84-89), so the encode-across modes keep the server's own (Hollanti passes it explicitly)
  c.num_parties = mode == 3 ? 2 : (NUM_PARTIES < 2 ? 2 : NUM_PARTIES);
  c.party_index = mode == 3 ? 1 : g.party;
  c.log_num_records = LOG_NUM_ENCODED_FILES;
  c.record_bytes = (uint32_t)ENCODED_FILE_SIZE_BYTES;
  c.num_rounds = rounds;
  c.is_byzantine = g.byzantine || (int)req.get_int("IsByzantine");
  if (pir_engine_create(&c, &g.eng) != PIR_OK) return std::string("engine: ") + pir_engine_last_error();
  if (ENCODE_ACROSS) {
    // the synthetic database of client.cpp:16-33, encoded across files on the GPU
    if (pir_engine_encode_across_dev(g.eng, nullptr, 0, (uint64_t)NUM_FILES, K) != PIR_OK)
      return std::string("encode: ") + pir_engine_last_error();
  } else {
    // the synthetic database of client.cpp:16-33, encoded within files (client.cpp:99-103) on
    // the GPU: no host copy of the database, no host encode under the lock
    if (pir_engine_encode_within_dev(g.eng, nullptr, 0, (uint64_t)NUM_FILES, FILE_SIZE_BYTES, K,
                                     g.party) != PIR_OK)
      return std::string("encode: ") + pir_engine_last_error();
  }
  g.mode = mode;
  g.nq = rounds;
  g.efs = ENCODED_FILE_SIZE_BYTES;
  g.p = NUM_PARTIES;
  g.t = T;
  g.cd_needed = NUM_CD_KEYS_NEEDED;
  g.num_files = (uint64_t)NUM_FILES;
  g.key_len = pir_engine_key_len(c.num_parties, c.log_num_records, c.num_rounds);
  return "";
}

// msgpack(error) then the search response map: Results [+ PartyIndex], the times
void write_search(Writer& w, const std::string& err, int nq, int efs, const std::vector<uint8_t>& out,
                  bool party_index, std::chrono::steady_clock::time_point t0,
                  std::chrono::system_clock::time_point recv) {
  err.empty() ? w.nil() : w.str(err);
  w.map(party_index ? 5 : 4);
  w.str("Results");
  if (err.empty()) {
    w.array((size_t)nq);
    for (int a = 0; a < nq; ++a) w.bin(out.data() + (size_t)a * efs, (size_t)efs);
  } else {
    w.array(0);
  }
  if (party_index) {
    w.str("PartyIndex");
    w.integer(g.party);
  }
  w.str("ServerLatency");
  w.integer(std::chrono::duration_cast<std::chrono::nanoseconds>(
                std::chrono::steady_clock::now() - t0).count());
  w.str("ReceiveTime");
  w.timestamp(recv);
  w.str("SendTime");
  w.timestamp(std::chrono::system_clock::now());
}

bool is_bytes(const MVal* v) { return v && (v->kind == MVal::BIN || v->kind == MVal::STR); }

void handle(SSL* ssl) {
  Stream in{ssl};
  for (;;) {
    uint8_t type;
    if (!in.byte(type)) return;  // EOF: the client is done
    MVal req = in.value();
    const auto recv = std::chrono::system_clock::now();
    const auto t0 = std::chrono::steady_clock::now();
    Writer w;
    std::string err;
    if (type == SETUP_REQUEST) {
      err = setup(req);
      err.empty() ? w.nil() : w.str(err);
      w.map(1);
      w.str("ServerLatency");
      w.integer(std::chrono::duration_cast<std::chrono::nanoseconds>(
                    std::chrono::steady_clock::now() - t0).count());
    } else if (type == TREE_SEARCH_REQUEST || type == MULTIPARTY_SEARCH_REQUEST ||
               type == HOLLANTI_SEARCH_REQUEST || type == CD732_SEARCH_REQUEST) {
      // tree.go:17-101, multiparty.go, hollanti.go, cd732.go
      const MVal* key = req.get("Key");
      std::vector<uint8_t> out;
      int nq = 0, efs = 0;  // this answer's shape, read under the lock with the engine
      {
        std::lock_guard<std::mutex> lk(g.mu);
        nq = g.nq;
        efs = g.efs;
        out.resize((size_t)nq * efs);
        const int want = type == TREE_SEARCH_REQUEST ? 0
                         : type == MULTIPARTY_SEARCH_REQUEST ? 1
                         : type == CD732_SEARCH_REQUEST ? 4 : 3;
        int rc = PIR_OK;
        if (!g.eng) {
          err = "query before setup";
        } else if (g.mode != want) {
          err = "request does not match the setup's mode";
        } else if (type == TREE_SEARCH_REQUEST) {
          if (!is_bytes(key) || (int)key->s.size() != g.key_len)  // the engine's own key length
            err = "bad key";
          else
            rc = pir_engine_answer(g.eng, (const uint8_t*)key->s.data(), out.data());
        } else if (type == MULTIPARTY_SEARCH_REQUEST) {  // the honest Thread path of multiparty.go:64
          if (!is_bytes(key))
            err = "bad key";
          else
            rc = pir_engine_answer_mp(g.eng, (const uint8_t*)key->s.data(), key->s.size(), g.p,
                                      g.t, 0, 1, out.data());
        } else if (type == CD732_SEARCH_REQUEST) {  // the Thread slices of cd732.go:61-76, XORed
          if (!is_bytes(key))
            err = "bad key";
          else
            rc = pir_engine_answer_cd(g.eng, (const uint8_t*)key->s.data(), key->s.size(),
                                      g.cd_needed, nq, 0, 1, out.data());
        } else {  // Key [][]byte: NUM_ROUNDS coefficient vectors of NUM_FILES bytes
          std::vector<const uint8_t*> ptrs;
          if (key && key->kind == MVal::ARR && (int)key->a.size() == nq)
            for (const MVal& v : key->a)
              if (is_bytes(&v) && v.s.size() == g.num_files) ptrs.push_back((const uint8_t*)v.s.data());
          if ((int)ptrs.size() != nq)
            err = "bad key";
          else
            rc = pir_engine_answer_coefs(g.eng, ptrs.data(), 0, g.num_files, out.data());
        }
        if (err.empty() && rc != PIR_OK) err = std::string("answer: ") + pir_engine_last_error();
      }
      write_search(w, err, nq, efs, out, type == TREE_SEARCH_REQUEST, t0, recv);
    } else if (type == TEST_REQUEST) {
      const MVal* msg = req.get("Msg");
      w.nil();
      w.map(1);
      w.str("Msg");
      w.str(msg && (msg->kind == MVal::STR || msg->kind == MVal::BIN) ? msg->s : "");
    } else {
      fprintf(stderr, "pir_serve: unknown request type %d\n", type);  // server.go:122
      return;
    }
    if (!send_all(ssl, w.b)) return;
  }
}

SSL_CTX* make_ctx(const char* cert, const char* key) {
  SSL_CTX* ctx = SSL_CTX_new(TLS_server_method());
  if (!ctx) return nullptr;
  if (cert && key) {
    if (SSL_CTX_use_certificate_chain_file(ctx, cert) != 1 ||
        SSL_CTX_use_PrivateKey_file(ctx, key, SSL_FILETYPE_PEM) != 1)
      return nullptr;
    return ctx;
  }
  // no certificate given: an ephemeral self-signed one (the reference's client skips
  // verification, network.go:27-30)
  EVP_PKEY* pk = EVP_EC_gen("P-256");
  X509* x = X509_new();
  if (!pk || !x) return nullptr;
  ASN1_INTEGER_set(X509_get_serialNumber(x), 1);
  X509_gmtime_adj(X509_getm_notBefore(x), 0);
  X509_gmtime_adj(X509_getm_notAfter(x), 7L * 24 * 3600);
  X509_set_pubkey(x, pk);
  X509_NAME* nm = X509_get_subject_name(x);
  X509_NAME_add_entry_by_txt(nm, "CN", MBSTRING_ASC, (const unsigned char*)"pir_serve", -1, -1, 0);
  X509_set_issuer_name(x, nm);
  if (!X509_sign(x, pk, EVP_sha256()) || SSL_CTX_use_certificate(ctx, x) != 1 ||
      SSL_CTX_use_PrivateKey(ctx, pk) != 1)
    return nullptr;
  X509_free(x);
  EVP_PKEY_free(pk);
  return ctx;
}

}  // namespace

int main(int argc, char** argv) {
  int port = 0;
  long max_conns = -1;
  const char *cert = nullptr, *key = nullptr;
  if (const char* d = getenv("PIR_DEVICE")) g.device = atoi(d);
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) { fprintf(stderr, "pir_serve: %s needs a value\n", a.c_str()); exit(2); }
      return argv[++i];
    };
    if (a == "--port") port = atoi(next());
    else if (a == "--party") g.party = atoi(next());
    else if (a == "--device") g.device = atoi(next());
    else if (a == "--byzantine") g.byzantine = atoi(next());
    else if (a == "--cert") cert = next();
    else if (a == "--key") key = next();
    else if (a == "--max-conns") max_conns = atol(next());
    else { fprintf(stderr, "pir_serve: unknown argument %s\n", a.c_str()); return 2; }
  }
  if (port <= 0 || g.party < 1) {
    fprintf(stderr, "usage: pir_serve --port P --party I [--cert C --key K] [--device D]\n");
    return 2;
  }
  signal(SIGPIPE, SIG_IGN);
  SSL_CTX* ctx = make_ctx(cert, key);
  if (!ctx) {
    ERR_print_errors_fp(stderr);
    return 1;
  }
  const int ls = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  addr.sin_addr.s_addr = htonl(INADDR_ANY);
  if (bind(ls, (sockaddr*)&addr, sizeof addr) != 0 || listen(ls, 64) != 0) {
    perror("pir_serve: bind/listen");
    return 1;
  }
  fprintf(stderr, "pir_serve: party %d listening on %d\n", g.party, port);
  std::vector<std::thread> workers;
  for (long n = 0; max_conns < 0 || n < max_conns; ++n) {
    const int fd = accept(ls, nullptr, nullptr);
    if (fd < 0) continue;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    workers.emplace_back([ctx, fd]() {  // one thread per connection (network.go:154-161)
      SSL* ssl = SSL_new(ctx);
      SSL_set_fd(ssl, fd);
      if (SSL_accept(ssl) == 1) {
        try {
          handle(ssl);
        } catch (const std::exception& ex) {
          fprintf(stderr, "pir_serve: %s\n", ex.what());
        }
        SSL_shutdown(ssl);
      }
      SSL_free(ssl);
      close(fd);
    });
  }
  for (auto& t : workers) t.join();
  {
    std::lock_guard<std::mutex> lk(g.mu);
    if (g.eng) pir_engine_destroy(g.eng);
  }
  SSL_CTX_free(ctx);
  return 0;
}
