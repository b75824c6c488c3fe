// C ABI of the native front-end (include/p265fe.h): NAL dispatch in stream order
// (dec.py:18-64, nalu.py:88-131), picture order count (8.3.1), output order, decoded
// picture hash SEI (D.2.20; nalu.py:130 raises on SEI), and parallel slice-data parsing of
// independent all-intra pictures on worker threads.
#include <algorithm>
#include <atomic>
#include <cstring>
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
    std::vector<size_t> nal_idx;            // slice segment NAL units, decode order
    std::vector<std::unique_ptr<SliceHeader>> hdrs;
    int poc = 0, nal_type = 0, output = 1, cvs = 0;
    int hash_type = P265FE_HASH_NONE;
    uint8_t hash[3][16] = {};
    int output_rank = -1;
};

bool is_irap(int t) { return t >= 16 && t <= 23; }
bool is_vcl_supported(int t) { return (t >= 0 && t <= 9) || (t >= 16 && t <= 21); }

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

}  // namespace

struct p265fe_decoder {
    std::vector<Nal> nals;
    std::vector<std::unique_ptr<PictureJob>> jobs;
    std::vector<PictureRecords> recs;
    std::string err;
};

static int set_err(p265fe_decoder* d, int code, const std::string& msg) {
    d->err = msg;
    return code;
}

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

void p265fe_destroy(p265fe_decoder* d) { delete d; }

const char* p265fe_last_error(p265fe_decoder* d) { return d ? d->err.c_str() : ""; }

int p265fe_decode(p265fe_decoder* d, const uint8_t* data, size_t size, int n_threads) {
    if (!d || (!data && size)) return P265FE_EINVAL;
    d->err.clear();
    d->jobs.clear();
    d->recs.clear();
    try {
        d->nals = split_nals(data, size);
        // ---- pass 1 (stream order): parameter sets, slice headers, POC, SEI ----
        std::shared_ptr<Sps> sps_tab[16];
        std::shared_ptr<Pps> pps_tab[64];
        std::shared_ptr<const Active> cached;
        const Sps* cached_sps = nullptr;
        const Pps* cached_pps = nullptr;
        PictureJob* cur = nullptr;
        const SliceHeader* prev_indep = nullptr;
        bool first_pic = true, after_eos = false;
        int prev_tid0_poc = 0, cvs = -1;
        bool no_rasl_output = false;
        for (size_t i = 0; i < d->nals.size(); ++i) {
            const Nal& nal = d->nals[i];
            if (nal.layer_id != 0) continue;
            BitReader br(nal.rbsp.data(), nal.rbsp.size());
            if (nal.type == 32) {
                parse_vps(br);
            } else if (nal.type == 33) {
                auto s = std::make_shared<Sps>(parse_sps(br));
                sps_tab[s->sps_id] = s;
            } else if (nal.type == 34) {
                auto p = std::make_shared<Pps>(parse_pps(br));
                pps_tab[p->pps_id] = p;
            } else if (nal.type == 36 || nal.type == 37) {   // end of sequence / bitstream
                after_eos = true;
                cur = nullptr;
            } else if (nal.type == 40 || nal.type == 39) {
                if (nal.type == 40 && cur) parse_picture_hash(nal.rbsp, cur->act->sps.chroma_format_idc, *cur);
            } else if (is_vcl_supported(nal.type)) {
                int first_in_pic = 0;
                int pps_id = peek_slice_pps_id(nal.rbsp, nal.type, &first_in_pic);
                if (pps_id > 63 || !pps_tab[pps_id]) bs_fail("slice refers to a missing PPS");
                const Pps* pps = pps_tab[pps_id].get();
                if (!sps_tab[pps->sps_id]) bs_fail("PPS refers to a missing SPS");
                const Sps* sps = sps_tab[pps->sps_id].get();
                if (first_in_pic) {
                    if (!cached || cached_sps != sps || cached_pps != pps) {
                        cached = activate(*sps, *pps);
                        cached_sps = sps;
                        cached_pps = pps;
                    }
                    d->jobs.push_back(std::make_unique<PictureJob>());
                    cur = d->jobs.back().get();
                    cur->act = cached;
                    cur->nal_type = nal.type;
                    prev_indep = nullptr;
                } else if (!cur) {
                    bs_fail("slice segment without the first slice segment of its picture");
                } else if (pps_id != cur->act->pps.pps_id) {
                    bs_fail("slice segments of one picture refer to different PPSs");
                }
                auto h = std::make_unique<SliceHeader>(parse_slice_header(br, nal.type, cur->act, prev_indep));
                if (!h->dependent) prev_indep = h.get();
                if (first_in_pic) {
                    // picture order count (8.3.1)
                    int max_lsb = 1 << cur->act->sps.log2_max_poc_lsb;
                    bool irap = is_irap(nal.type);
                    if (irap) {
                        no_rasl_output = (nal.type >= 16 && nal.type <= 20) || first_pic || after_eos;
                        if (no_rasl_output) ++cvs;
                    } else if (first_pic) {
                        bs_fail("stream does not start with an IRAP picture");
                    }
                    int lsb = (nal.type == 19 || nal.type == 20) ? 0 : h->poc_lsb;
                    int msb;
                    if (irap && no_rasl_output) {
                        msb = 0;
                    } else {
                        int prev_lsb = prev_tid0_poc & (max_lsb - 1);
                        int prev_msb = prev_tid0_poc - prev_lsb;
                        if (lsb < prev_lsb && prev_lsb - lsb >= max_lsb / 2) msb = prev_msb + max_lsb;
                        else if (lsb > prev_lsb && lsb - prev_lsb > max_lsb / 2) msb = prev_msb - max_lsb;
                        else msb = prev_msb;
                    }
                    cur->poc = msb + lsb;
                    cur->cvs = cvs;
                    bool rasl = nal.type == 8 || nal.type == 9, radl = nal.type == 6 || nal.type == 7;
                    bool slnr = nal.type <= 14 && (nal.type % 2) == 0;
                    if (nal.temporal_id == 0 && !rasl && !radl && !slnr) prev_tid0_poc = cur->poc;
                    cur->output = (rasl && no_rasl_output) ? 0 : h->pic_output_flag;
                    first_pic = false;
                    after_eos = false;
                }
                cur->nal_idx.push_back(i);
                cur->hdrs.push_back(std::move(h));
            }
        }
        // output order: by (coded video sequence, POC) among output pictures
        std::vector<PictureJob*> outv;
        for (auto& j : d->jobs)
            if (j->output) outv.push_back(j.get());
        std::stable_sort(outv.begin(), outv.end(), [](const PictureJob* a, const PictureJob* b) {
            return a->cvs != b->cvs ? a->cvs < b->cvs : a->poc < b->poc;
        });
        for (size_t r = 0; r < outv.size(); ++r) outv[r]->output_rank = (int)r;

        // ---- pass 2: slice data of independent pictures on worker threads ----
        size_t np = d->jobs.size();
        d->recs.resize(np);
        int nt = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
        nt = (int)std::min<size_t>((size_t)nt, std::max<size_t>(np, 1));
        std::atomic<size_t> next{0};
        std::mutex emu;
        int first_code = 0;
        std::string first_msg;
        size_t first_pic_err = (size_t)-1;
        auto worker = [&]() {
            for (;;) {
                size_t k = next.fetch_add(1);
                if (k >= np) return;
                PictureJob& j = *d->jobs[k];
                std::vector<SliceRef> sl;
                for (size_t s = 0; s < j.nal_idx.size(); ++s) {
                    const Nal& nal = d->nals[j.nal_idx[s]];
                    sl.push_back(SliceRef{j.hdrs[s].get(), nal.rbsp.data(), nal.rbsp.size()});
                }
                int code = 0;
                std::string msg;
                try {
                    decode_picture(*j.act, sl, d->recs[k]);
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
                        first_msg = "picture " + std::to_string(k) + ": " + msg;
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
        if (first_code) return set_err(d, first_code, first_msg);
        return (int)np;
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

int p265fe_picture(p265fe_decoder* d, int i, p265fe_picture_info* out) {
    if (!d || !out || i < 0 || (size_t)i >= d->jobs.size() || (size_t)i >= d->recs.size()) return P265FE_EINVAL;
    const PictureJob& j = *d->jobs[i];
    const PictureRecords& r = d->recs[i];
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
    out->n_slices = (uint16_t)j.nal_idx.size();
    out->n_cus = r.n_cus;
    std::memcpy(out->hash, j.hash, sizeof(out->hash));
    return P265FE_OK;
}

}  // extern "C"
