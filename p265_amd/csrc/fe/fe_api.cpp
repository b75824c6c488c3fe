// C ABI of the native front-end (include/p265fe.h): NAL dispatch in stream order
// (dec.py:18-64, nalu.py:88-131), access-unit assembly, picture order count (8.3.1),
// decoded picture hash SEI (D.2.20; nalu.py:130 raises on SEI), and parallel slice-data
// parsing of independent all-intra pictures on worker threads.  Streams can be fed in
// arbitrary chunks (p265fe_feed / p265fe_take): parameter sets, POC state, the picture
// being assembled and an incomplete trailing NAL unit carry over between calls.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/p265fe.h"
#include "fe_picture.h"
#include "fe_ps.h"

using namespace p265fe;

namespace {

struct PictureJob {
    std::shared_ptr<const Active> act;
    std::vector<Nal> slices;                // slice segment NAL units, decode order
    std::vector<std::unique_ptr<SliceHeader>> hdrs;
    int poc = 0, nal_type = 0, output = 1, cvs = 0;
    int hash_type = P265FE_HASH_NONE;
    uint8_t hash[3][16] = {};
    int output_rank = -1;
};

bool is_irap(int t) { return t >= 16 && t <= 23; }
bool is_vcl_supported(int t) { return (t >= 0 && t <= 9) || (t >= 16 && t <= 21); }
// NAL unit types that start a new access unit (7.4.2.4.4) besides a first slice segment
bool starts_access_unit(int t) { return (t >= 32 && t <= 35) || t == 39 || (t >= 41 && t <= 44) || (t >= 48 && t <= 55); }

// decoded_picture_hash (D.2.20) from an SEI RBSP (7.3.5); returns true if found
bool parse_picture_hash(const std::vector<uint8_t>& rbsp, int chroma_format_idc, PictureJob& job) {
    size_t p = 0, n = rbsp.size();
    while (p < n) {
        if (p + 1 >= n && rbsp[p] == 0x80) break;   // rbsp_trailing_bits
        int type = 0, size = 0;
        while (p < n && rbsp[p] == 0xFF) { type += 255; ++p; }
        if (p >= n) return false;
        type += rbsp[p++];
        while (p < n && rbsp[p] == 0xFF) { size += 255; ++p; }
        if (p >= n) return false;
        size += rbsp[p++];
        if (p + (size_t)size > n) return false;
        if (type == 132 && size >= 1) {
            int ht = rbsp[p];
            int ncomp = chroma_format_idc == 0 ? 1 : 3;
            int len = ht == 0 ? 16 : ht == 1 ? 2 : ht == 2 ? 4 : -1;
            if (len > 0 && size >= 1 + ncomp * len) {
                job.hash_type = ht;
                for (int c = 0; c < ncomp; ++c) std::memcpy(job.hash[c], &rbsp[p + 1 + (size_t)c * len], (size_t)len);
                return true;
            }
        }
        p += (size_t)size;
    }
    return false;
}

// Stream-order state that survives between p265fe_feed calls.
struct StreamState {
    std::shared_ptr<Sps> sps_tab[16];
    std::shared_ptr<Pps> pps_tab[64];
    std::shared_ptr<const Active> cached;
    const Sps* cached_sps = nullptr;
    const Pps* cached_pps = nullptr;
    std::unique_ptr<PictureJob> cur;          // access unit being assembled
    const SliceHeader* prev_indep = nullptr;  // into cur->hdrs
    bool first_pic = true, after_eos = false, no_rasl_output = false;
    int prev_tid0_poc = 0, cvs = -1;
    std::vector<uint8_t> tail;                // from the last start code of the previous feed
    std::vector<std::unique_ptr<PictureJob>> complete;   // assembled, slice data not parsed yet
};

}  // namespace

struct p265fe_pictures {
    std::vector<std::unique_ptr<PictureJob>> jobs;
    std::vector<PictureRecords> recs;
};

// Asynchronous slice-data parsing (P265FE_ASYNC): complete access units go to persistent workers;
// the decoder hands them out in decode order as the prefix of parsed pictures grows, so parsing of
// later chunks overlaps the stragglers of earlier ones (no per-chunk join).
struct AsyncParser {
    struct Slot {
        std::unique_ptr<PictureJob> job;
        PictureRecords rec;
        int state = 0;                          // 0 queued, 1 parsing, 2 done
        int code = 0;
        std::string msg;
    };
    std::mutex m;
    std::condition_variable cv_work, cv_done;
    std::deque<std::unique_ptr<Slot>> slots;    // submitted, not yet taken, decode order
    size_t next_work = 0;                       // slots[0 .. next_work) handed to a worker
    uint64_t base = 0;                          // decode index of slots[0]
    std::vector<std::thread> workers;
    bool quit = false;

    void start(int n) {
        if (!workers.empty()) return;
        for (int t = 0; t < std::max(1, n); ++t) workers.emplace_back([this] { run(); });
    }
    void run() {
        for (;;) {
            Slot* sl = nullptr;
            uint64_t idx = 0;
            {
                std::unique_lock<std::mutex> g(m);
                cv_work.wait(g, [&] { return quit || next_work < slots.size(); });
                if (quit) return;
                sl = slots[next_work].get();
                idx = base + next_work;
                ++next_work;
                sl->state = 1;
            }
            PictureJob& j = *sl->job;
            std::vector<SliceRef> sr;
            for (size_t k = 0; k < j.slices.size(); ++k)
                sr.push_back(SliceRef{j.hdrs[k].get(), j.slices[k].rbsp.data(), j.slices[k].rbsp.size()});
            int code = 0;
            std::string msg;
            try {
                decode_picture(*j.act, sr, sl->rec);
            } catch (const Unsupported& e) {
                code = P265FE_EUNSUPPORTED; msg = e.what();
            } catch (const BitstreamError& e) {
                code = P265FE_EBITSTREAM; msg = e.what();
            } catch (const std::bad_alloc&) {
                code = P265FE_ENOMEM; msg = "out of memory";
            } catch (const std::exception& e) {
                code = P265FE_EBITSTREAM; msg = e.what();
            }
            {
                std::lock_guard<std::mutex> g(m);
                sl->code = code;
                if (code) sl->msg = "picture " + std::to_string(idx) + ": " + msg;
                sl->state = 2;
            }
            cv_done.notify_all();
        }
    }
    void submit(std::vector<std::unique_ptr<PictureJob>>& jobs) {
        {
            std::lock_guard<std::mutex> g(m);
            for (auto& j : jobs) {
                auto sl = std::make_unique<Slot>();
                sl->job = std::move(j);
                slots.push_back(std::move(sl));
            }
        }
        jobs.clear();
        cv_work.notify_all();
    }
    size_t done_prefix_locked() const {
        size_t k = 0;
        while (k < slots.size() && slots[k]->state == 2) ++k;
        return k;
    }
    ~AsyncParser() {
        {
            std::lock_guard<std::mutex> g(m);
            quit = true;
        }
        cv_work.notify_all();
        for (auto& t : workers) t.join();
    }
};

struct p265fe_decoder {
    StreamState st;
    p265fe_pictures ready;                    // parsed, not yet taken
    p265fe_pictures* last = nullptr;          // result of p265fe_decode (p265fe_picture)
    std::unique_ptr<AsyncParser> async;       // P265FE_ASYNC feeds
    std::string err;
};

static int set_err(p265fe_decoder* d, int code, const std::string& msg) {
    d->err = msg;
    return code;
}

namespace {

void finish_current(StreamState& st) {
    if (st.cur) st.complete.push_back(std::move(st.cur));
    st.cur.reset();
    st.prev_indep = nullptr;
}

// Stream-order processing of one complete NAL unit.
void process_nal(StreamState& st, Nal&& nal) {
    if (nal.layer_id != 0) return;
    const int t = nal.type;
    if (starts_access_unit(t)) finish_current(st);
    BitReader br(nal.rbsp.data(), nal.rbsp.size());
    if (t == 32) {
        parse_vps(br);
    } else if (t == 33) {
        auto s = std::make_shared<Sps>(parse_sps(br));
        st.sps_tab[s->sps_id] = s;
    } else if (t == 34) {
        auto p = std::make_shared<Pps>(parse_pps(br));
        st.pps_tab[p->pps_id] = p;
    } else if (t == 36 || t == 37) {                    // end of sequence / bitstream
        finish_current(st);
        st.after_eos = true;
    } else if (t == 40) {                               // suffix SEI: belongs to the current picture
        if (st.cur) parse_picture_hash(nal.rbsp, st.cur->act->sps.chroma_format_idc, *st.cur);
    } else if (is_vcl_supported(t)) {
        int first_in_pic = 0;
        int pps_id = peek_slice_pps_id(nal.rbsp, t, &first_in_pic);
        if (pps_id > 63 || !st.pps_tab[pps_id]) bs_fail("slice refers to a missing PPS");
        const Pps* pps = st.pps_tab[pps_id].get();
        if (!st.sps_tab[pps->sps_id]) bs_fail("PPS refers to a missing SPS");
        const Sps* sps = st.sps_tab[pps->sps_id].get();
        if (first_in_pic) {
            finish_current(st);
            if (!st.cached || st.cached_sps != sps || st.cached_pps != pps) {
                st.cached = activate(*sps, *pps);
                st.cached_sps = sps;
                st.cached_pps = pps;
            }
            st.cur = std::make_unique<PictureJob>();
            st.cur->act = st.cached;
            st.cur->nal_type = t;
        } else if (!st.cur) {
            bs_fail("slice segment without the first slice segment of its picture");
        } else if (pps_id != st.cur->act->pps.pps_id) {
            bs_fail("slice segments of one picture refer to different PPSs");
        }
        PictureJob& cur = *st.cur;
        auto h = std::make_unique<SliceHeader>(parse_slice_header(br, t, cur.act, st.prev_indep));
        if (!h->dependent) st.prev_indep = h.get();
        if (first_in_pic) {
            // picture order count (8.3.1)
            int max_lsb = 1 << cur.act->sps.log2_max_poc_lsb;
            bool irap = is_irap(t);
            if (irap) {
                st.no_rasl_output = (t >= 16 && t <= 20) || st.first_pic || st.after_eos;
                if (st.no_rasl_output) ++st.cvs;
            } else if (st.first_pic) {
                bs_fail("stream does not start with an IRAP picture");
            }
            int lsb = (t == 19 || t == 20) ? 0 : h->poc_lsb;
            int msb;
            if (irap && st.no_rasl_output) {
                msb = 0;
            } else {
                int prev_lsb = st.prev_tid0_poc & (max_lsb - 1);
                int prev_msb = st.prev_tid0_poc - prev_lsb;
                if (lsb < prev_lsb && prev_lsb - lsb >= max_lsb / 2) msb = prev_msb + max_lsb;
                else if (lsb > prev_lsb && lsb - prev_lsb > max_lsb / 2) msb = prev_msb - max_lsb;
                else msb = prev_msb;
            }
            cur.poc = msb + lsb;
            cur.cvs = st.cvs;
            bool rasl = t == 8 || t == 9, radl = t == 6 || t == 7;
            bool slnr = t <= 14 && (t % 2) == 0;
            if (nal.temporal_id == 0 && !rasl && !radl && !slnr) st.prev_tid0_poc = cur.poc;
            cur.output = (rasl && st.no_rasl_output) ? 0 : h->pic_output_flag;
            st.first_pic = false;
            st.after_eos = false;
        }
        cur.hdrs.push_back(std::move(h));
        cur.slices.push_back(std::move(nal));
    }
}

// Parse the slice data of the complete pictures on worker threads; append to `out`.
int parse_pictures(std::vector<std::unique_ptr<PictureJob>>& jobs, p265fe_pictures& out, int n_threads,
                   std::string& err) {
    size_t np = jobs.size(), base = out.recs.size();
    out.recs.resize(base + np);
    int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = (int)std::min<size_t>((size_t)nt, std::max<size_t>(np, 1));
    std::atomic<size_t> next{0};
    std::mutex emu;
    int first_code = 0;
    size_t first_pic_err = (size_t)-1;
    auto worker = [&]() {
        for (;;) {
            size_t k = next.fetch_add(1);
            if (k >= np) return;
            PictureJob& j = *jobs[k];
            std::vector<SliceRef> sl;
            for (size_t s = 0; s < j.slices.size(); ++s)
                sl.push_back(SliceRef{j.hdrs[s].get(), j.slices[s].rbsp.data(), j.slices[s].rbsp.size()});
            int code = 0;
            std::string msg;
            try {
                decode_picture(*j.act, sl, out.recs[base + k]);
            } catch (const Unsupported& e) {
                code = P265FE_EUNSUPPORTED; msg = e.what();
            } catch (const BitstreamError& e) {
                code = P265FE_EBITSTREAM; msg = e.what();
            } catch (const std::bad_alloc&) {
                code = P265FE_ENOMEM; msg = "out of memory";
            } catch (const std::exception& e) {
                code = P265FE_EBITSTREAM; msg = e.what();
            }
            if (code) {
                std::lock_guard<std::mutex> g(emu);
                if (k < first_pic_err) {
                    first_pic_err = k;
                    first_code = code;
                    err = "picture " + std::to_string(base + k) + ": " + msg;
                }
            }
        }
    };
    if (nt <= 1) {
        worker();
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back(worker);
        for (auto& t : th) t.join();
    }
    if (first_code) {
        out.recs.resize(base);
        jobs.clear();
        return first_code;
    }
    for (auto& j : jobs) out.jobs.push_back(std::move(j));
    jobs.clear();
    return 0;
}

void fill_info(const PictureJob& j, const PictureRecords& r, p265fe_picture_info* out) {
    const Sps& s = j.act->sps;
    const Pps& p = j.act->pps;
    std::memset(out, 0, sizeof(*out));
    p265r_params& pr = out->params;
    pr.version = P265R_ABI_VERSION;
    pr.pic_width = (uint16_t)s.width;
    pr.pic_height = (uint16_t)s.height;
    pr.chroma_format_idc = (uint8_t)s.chroma_format_idc;
    pr.bit_depth_luma = (uint8_t)s.bit_depth_y;
    pr.bit_depth_chroma = (uint8_t)s.bit_depth_c;
    pr.ctb_log2_size = (uint8_t)s.log2_ctb;
    pr.min_tb_log2_size = (uint8_t)s.log2_min_tb;
    pr.max_tb_log2_size = (uint8_t)s.log2_max_tb;
    pr.strong_intra_smoothing = (uint8_t)s.strong_intra_smoothing;
    pr.constrained_intra_pred = (uint8_t)p.constrained_intra_pred;
    pr.sample_adaptive_offset = (uint8_t)s.sao;
    pr.loop_filter_across_tiles = (uint8_t)p.loop_filter_across_tiles;
    pr.scaling_list_enabled = (uint8_t)s.scaling_list_enabled;
    pr.pps_cb_qp_offset = (int8_t)p.cb_qp_offset;
    pr.pps_cr_qp_offset = (int8_t)p.cr_qp_offset;
    out->ctus = r.ctus.data();
    out->n_ctus = (uint32_t)r.ctus.size();
    out->tbs = r.tbs.data();
    out->n_tbs = (uint32_t)r.tbs.size();
    out->coef = r.coef.data();
    out->n_coef = r.coef.size();
    out->nofilter = r.nofilter.empty() ? nullptr : r.nofilter.data();
    out->poc = j.poc;
    out->output_rank = j.output_rank;
    int sw = s.chroma_format_idc == 1 || s.chroma_format_idc == 2 ? 2 : 1;
    int sh = s.chroma_format_idc == 1 ? 2 : 1;
    out->crop_left = (uint16_t)(sw * s.conf_left);
    out->crop_right = (uint16_t)(sw * s.conf_right);
    out->crop_top = (uint16_t)(sh * s.conf_top);
    out->crop_bottom = (uint16_t)(sh * s.conf_bottom);
    out->nal_unit_type = (uint8_t)j.nal_type;
    out->hash_type = (int8_t)j.hash_type;
    out->n_slices = (uint16_t)j.slices.size();
    out->n_cus = r.n_cus;
    std::memcpy(out->hash, j.hash, sizeof(out->hash));
    out->cvs_id = j.cvs;
    out->scaling_factors = s.scaling_list_enabled ? j.act->scaling_factor.data() : nullptr;
    out->max_num_reorder = (uint8_t)s.max_num_reorder;
    out->output_flag = (uint8_t)(j.output ? 1 : 0);
}

}  // namespace

extern "C" {

uint32_t p265fe_abi_version(void) { return P265FE_ABI_VERSION; }

int p265fe_create(p265fe_decoder** out) {
    if (!out) return P265FE_EINVAL;
    try {
        *out = new p265fe_decoder();
    } catch (...) {
        return P265FE_ENOMEM;
    }
    return P265FE_OK;
}

void p265fe_destroy(p265fe_decoder* d) {
    if (!d) return;
    delete d->last;
    delete d;
}

const char* p265fe_last_error(p265fe_decoder* d) { return d ? d->err.c_str() : ""; }

int p265fe_feed(p265fe_decoder* d, const uint8_t* data, size_t size, int n_threads, int flags) {
    if (!d || (!data && size) || (flags & ~(P265FE_FLUSH | P265FE_ASYNC))) return P265FE_EINVAL;
    const bool async = (flags & P265FE_ASYNC) != 0;
    if (async != (d->async != nullptr) && (d->async || !d->ready.jobs.empty())) return P265FE_EINVAL;   // no mixing
    d->err.clear();
    StreamState& st = d->st;
    try {
        std::vector<uint8_t> buf;
        buf.reserve(st.tail.size() + size);
        buf.insert(buf.end(), st.tail.begin(), st.tail.end());
        if (size) buf.insert(buf.end(), data, data + size);
        st.tail.clear();
        size_t cut = buf.size();
        if (!(flags & P265FE_FLUSH)) {
            // the NAL unit after the last start code may continue in the next chunk
            cut = 0;
            for (size_t k = buf.size() >= 3 ? buf.size() - 2 : 0; k-- > 0;)
                if (buf[k] == 0 && buf[k + 1] == 0 && buf[k + 2] == 1) { cut = k; break; }
            st.tail.assign(buf.begin() + (long)cut, buf.end());
        }
        std::vector<Nal> nals = split_nals(buf.data(), cut);
        for (auto& nal : nals) process_nal(st, std::move(nal));
        if (flags & P265FE_FLUSH) finish_current(st);
        if (async) {
            if (!d->async) d->async = std::make_unique<AsyncParser>();
            d->async->start(n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency()));
            d->async->submit(st.complete);
            std::lock_guard<std::mutex> g(d->async->m);
            return (int)d->async->slots.size();
        }
        int rc = parse_pictures(st.complete, d->ready, n_threads, d->err);
        if (rc) return rc;
        return (int)d->ready.jobs.size();
    } catch (const Unsupported& e) {
        return set_err(d, P265FE_EUNSUPPORTED, e.what());
    } catch (const BitstreamError& e) {
        return set_err(d, P265FE_EBITSTREAM, e.what());
    } catch (const std::bad_alloc&) {
        return set_err(d, P265FE_ENOMEM, "out of memory");
    } catch (const std::exception& e) {
        return set_err(d, P265FE_EBITSTREAM, e.what());
    }
}

int p265fe_take(p265fe_decoder* d, p265fe_pictures** out) {
    if (!d || !out) return P265FE_EINVAL;
    *out = nullptr;
    auto* set = new (std::nothrow) p265fe_pictures();
    if (!set) return P265FE_ENOMEM;
    if (d->async) {                             // the parsed prefix, decode order; stop at an error
        AsyncParser& a = *d->async;
        std::lock_guard<std::mutex> g(a.m);
        const size_t n = a.done_prefix_locked();
        size_t k = 0;
        for (; k < n; ++k) {
            if (a.slots[k]->code) break;
            set->jobs.push_back(std::move(a.slots[k]->job));
            set->recs.push_back(std::move(a.slots[k]->rec));
        }
        const int code = k < n ? a.slots[k]->code : 0;
        if (code) d->err = a.slots[k]->msg;
        for (size_t i = 0; i < k; ++i) a.slots.pop_front();
        a.base += k;
        a.next_work -= k;
        if (code && set->jobs.empty()) {
            // the failed picture is reported ONCE and dropped: later takes hand out the pictures
            // after it (a caller resyncs at the next IRAP), and feed's pending count drains
            a.slots.pop_front();
            a.base += 1;
            a.next_work -= 1;
            delete set;
            return code;
        }
        *out = set;
        return (int)set->jobs.size();
    }
    set->jobs = std::move(d->ready.jobs);
    set->recs = std::move(d->ready.recs);
    d->ready.jobs.clear();
    d->ready.recs.clear();
    *out = set;
    return (int)set->jobs.size();
}

int p265fe_wait(p265fe_decoder* d, int all) {
    if (!d) return P265FE_EINVAL;
    if (!d->async) return (int)d->ready.jobs.size();
    AsyncParser& a = *d->async;
    std::unique_lock<std::mutex> g(a.m);
    a.cv_done.wait(g, [&] {
        const size_t n = a.done_prefix_locked();
        if (all) return n == a.slots.size();
        return a.slots.empty() || n > 0;
    });
    return (int)a.done_prefix_locked();
}

int p265fe_pictures_get(const p265fe_pictures* set, int i, p265fe_picture_info* out) {
    if (!set || !out || i < 0 || (size_t)i >= set->jobs.size()) return P265FE_EINVAL;
    fill_info(*set->jobs[i], set->recs[i], out);
    return P265FE_OK;
}

void p265fe_pictures_free(p265fe_pictures* set) { delete set; }

int p265fe_decode(p265fe_decoder* d, const uint8_t* data, size_t size, int n_threads) {
    if (!d || (!data && size)) return P265FE_EINVAL;
    d->async.reset();
    d->st = StreamState();
    d->ready = p265fe_pictures();
    delete d->last;
    d->last = nullptr;
    int n = p265fe_feed(d, data, size, n_threads, P265FE_FLUSH);
    if (n < 0) return n;
    p265fe_pictures* set = nullptr;
    int rc = p265fe_take(d, &set);
    if (rc < 0) return rc;
    // output order of the whole stream: by (coded video sequence, POC) among output pictures
    std::vector<PictureJob*> outv;
    for (auto& j : set->jobs)
        if (j->output) outv.push_back(j.get());
    std::stable_sort(outv.begin(), outv.end(), [](const PictureJob* a, const PictureJob* b) {
        return a->cvs != b->cvs ? a->cvs < b->cvs : a->poc < b->poc;
    });
    for (size_t r = 0; r < outv.size(); ++r) outv[r]->output_rank = (int)r;
    d->last = set;
    return (int)set->jobs.size();
}

int p265fe_picture(p265fe_decoder* d, int i, p265fe_picture_info* out) {
    if (!d || !d->last) return P265FE_EINVAL;
    return p265fe_pictures_get(d->last, i, out);
}

}  // extern "C"
