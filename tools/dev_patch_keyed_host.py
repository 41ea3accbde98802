"""One-off source patch (kept for the record): host side of keyed batch MSMs."""
p = '/root/repo/narwhal_amd/csrc/nwv_host.hip'
s = open(p).read()


def rep(old, new, count=1):
    global s
    assert s.count(old) >= 1, old[:80]
    s = s.replace(old, new, count)


rep('''    DevBuf m_scal, m_partial, m_state, m_pts, m_digits, m_cnt, m_tiles, m_entries, m_kstart, m_hpart,
        m_bsum, m_wsum;
    void release() {
        for (DevBuf* b : {&pk, &sig, &msg, &off, &len, &kbuf, &flags, &tables, &verdict, &m_scal,
                          &m_partial, &m_state, &m_pts, &m_digits, &m_cnt, &m_tiles, &m_entries,
                          &m_kstart, &m_hpart, &m_bsum, &m_wsum})
            b->release();
    }''', '''    DevBuf m_scal, m_partial, m_state, m_pts, m_digits, m_cnt, m_tiles, m_entries, m_kstart, m_hpart,
        m_bsum, m_wsum;
    // keyed batches: distinct keys (m x 32), CSR of signatures by key, per-signature z_i k_i
    DevBuf keys, koff, ksig, m_ascal;
    size_t nkeys_distinct = 0;  // 0: every signature is its own A point
    void release() {
        for (DevBuf* b : {&pk, &sig, &msg, &off, &len, &kbuf, &flags, &tables, &verdict, &m_scal,
                          &m_partial, &m_state, &m_pts, &m_digits, &m_cnt, &m_tiles, &m_entries,
                          &m_kstart, &m_hpart, &m_bsum, &m_wsum, &keys, &koff, &ksig, &m_ascal})
            b->release();
        nkeys_distinct = 0;
    }''')

rep('''// Window layout and work decomposition of one batch MSM over np = 2n + 1 points.
struct MsmPlan {''', '''// Window layout and work decomposition of one batch MSM over np = na + 1 + n points (na A
// points: n, or the m distinct keys of a keyed batch).
struct MsmPlan {''')
rep('''    uint64_t np = 0, cnt_len = 0, max_entries = 0, nseg = 0;
};''', '''    uint64_t np = 0, na = 0, cnt_len = 0, max_entries = 0, nseg = 0;
};''')
rep('''MsmPlan msm_plan(size_t n) {
    MsmPlan p;
    p.np = 2 * (uint64_t)n + 1;''', '''MsmPlan msm_plan(size_t n, size_t na) {
    MsmPlan p;
    p.na = na;
    p.np = (uint64_t)na + 1 + n;''')
rep('''        const double entries = (double)(n + 1) * L.nw + (double)n * L.nw_z;''',
    '''        const double entries = (double)(na + 1) * L.nw + (double)n * L.nw_z;''')
rep('''    p.max_entries = (uint64_t)(n + 1) * p.lay.nw + (uint64_t)n * p.lay.nw_z;''',
    '''    p.max_entries = (uint64_t)(na + 1) * p.lay.nw + (uint64_t)n * p.lay.nw_z;''')
rep('''    if ((rc = b.m_scal.ensure(32 * p.np + 32)) ||''', '''    if ((rc = b.m_scal.ensure(64)) || (b.nkeys_distinct && (rc = b.m_ascal.ensure(32 * n + 32))) ||''')

rep('''    if (n == 0) return NWV_OK;
    const MsmPlan p = msm_plan(n);''', '''    if (n == 0) return NWV_OK;
    const size_t na = b.nkeys_distinct ? b.nkeys_distinct : n;
    const MsmPlan p = msm_plan(n, na);''')
rep('''    hipLaunchKernelGGL(k_msm_scalars, dim3(nblk), dim3(256), 0, stream, (uint64_t)n, b.pk.as<uint8_t>(),
                       b.sig.as<uint8_t>(), b.msg.as<uint8_t>(), b.off.as<uint64_t>(), b.len.as<uint32_t>(),
                       seed, p.lay, b.m_scal.as<uint32_t>(), digits, b.m_partial.as<uint32_t>(), state);''',
    '''    const int keyed = b.nkeys_distinct ? 1 : 0;
    hipLaunchKernelGGL(k_msm_scalars, dim3(nblk), dim3(256), 0, stream, (uint64_t)n, (uint64_t)na, keyed,
                       b.pk.as<uint8_t>(), b.sig.as<uint8_t>(), b.msg.as<uint8_t>(), b.off.as<uint64_t>(),
                       b.len.as<uint32_t>(), seed, p.lay, b.m_ascal.as<uint32_t>(), digits,
                       b.m_partial.as<uint32_t>(), state);
    if (keyed)
        hipLaunchKernelGGL(k_msm_keysum, dim3((unsigned)na), dim3(256), 0, stream, (uint64_t)n, (uint64_t)na,
                           p.lay, b.koff.as<uint32_t>(), b.ksig.as<uint32_t>(), b.m_ascal.as<uint32_t>(), digits);''')
rep('''    hipLaunchKernelGGL(k_msm_bscalar, dim3(1), dim3(256), 0, stream, (uint64_t)n, (uint32_t)nblk, p.lay,''',
    '''    hipLaunchKernelGGL(k_msm_bscalar, dim3(1), dim3(256), 0, stream, (uint64_t)n, (uint64_t)na, (uint32_t)nblk,
                       p.lay,''')
rep('''    const size_t waves = (n + 63) / 64;
    hipLaunchKernelGGL(k_msm_points, dim3((unsigned)((2 * 64 * waves + 255) / 256)), dim3(256), 0, stream,
                       (uint64_t)n, b.pk.as<uint8_t>(), b.sig.as<uint8_t>(), b.m_pts.as<uint32_t>(), state);''',
    '''    const size_t waves = (n + 63) / 64 + (na + 63) / 64;
    hipLaunchKernelGGL(k_msm_points, dim3((unsigned)((64 * waves + 255) / 256)), dim3(256), 0, stream,
                       (uint64_t)n, (uint64_t)na, keyed ? b.keys.as<uint8_t>() : b.pk.as<uint8_t>(),
                       b.sig.as<uint8_t>(), b.m_pts.as<uint32_t>(), state);''')
rep('''    hipLaunchKernelGGL(k_msm_hist, gsort, dim3(256), lds_nb, stream, (uint64_t)n, p.lay, p.chunk_pts,''',
    '''    hipLaunchKernelGGL(k_msm_hist, gsort, dim3(256), lds_nb, stream, (uint64_t)n, (uint64_t)na, p.lay, p.chunk_pts,''')
rep('''    hipLaunchKernelGGL(k_msm_scatter, gsort, dim3(256), lds_nb, stream, (uint64_t)n, p.lay,''',
    '''    hipLaunchKernelGGL(k_msm_scatter, gsort, dim3(256), lds_nb, stream, (uint64_t)n, (uint64_t)na, p.lay,''')

# keyed staging helper: after ed_stage, set the key list and CSR (host-built)
rep('''bool verdicts_all_valid(const uint64_t* bits, size_t n) {''', '''// Keyed staging: signature i of [lo, hi) is by keys[key_idx[i]].  The distinct keys that occur
// in the range are renumbered densely, uploaded with the CSR of signatures per key, and pk is
// expanded per signature (the per-signature fallback reads it).  Call after ed_stage with
// pk == nullptr... i.e. ed_stage_keyed does both.
int ed_stage_keyed(Device& d, EdBuffers& b, size_t lo, size_t hi, size_t n_keys, const uint8_t* keys,
                   const uint32_t* key_idx, const uint8_t* sig, const uint8_t* msg_base,
                   const uint64_t* msg_off, const uint32_t* msg_len) {
    const size_t n = hi - lo;
    std::vector<uint32_t> local(n_keys, UINT32_MAX), cnt;
    std::vector<uint32_t> kid(n);
    std::vector<uint8_t> klist, pk(32 * n + 16);
    for (size_t i = 0; i < n; i++) {
        const uint32_t g = key_idx[lo + i];
        if (g >= n_keys) return set_err(NWV_ERR_ARG, "key index out of range");
        if (local[g] == UINT32_MAX) {
            local[g] = (uint32_t)cnt.size();
            cnt.push_back(0);
            klist.insert(klist.end(), keys + 32 * (size_t)g, keys + 32 * (size_t)g + 32);
        }
        kid[i] = local[g];
        cnt[kid[i]]++;
        std::memcpy(pk.data() + 32 * i, keys + 32 * (size_t)g, 32);
    }
    const size_t m = cnt.size();
    std::vector<uint32_t> koff(m + 1, 0), ksig(n), cur;
    for (size_t k = 0; k < m; k++) koff[k + 1] = koff[k] + cnt[k];
    cur.assign(koff.begin(), koff.end() - 1);
    for (size_t i = 0; i < n; i++) ksig[cur[kid[i]]++] = (uint32_t)i;
    int rc = ed_stage(d, b, 0, n, pk.data(), sig + 64 * lo, msg_base, msg_off + lo, msg_len + lo);
    if (rc) return rc;
    if ((rc = b.keys.ensure(32 * m + 32)) || (rc = b.koff.ensure(4 * m + 8)) || (rc = b.ksig.ensure(4 * n + 8)))
        return rc;
    if (m) {
        NWV_HIP(hipMemcpyAsync(b.keys.p, klist.data(), 32 * m, hipMemcpyHostToDevice, d.stream));
        NWV_HIP(hipMemcpyAsync(b.koff.p, koff.data(), 4 * (m + 1), hipMemcpyHostToDevice, d.stream));
    }
    if (n) NWV_HIP(hipMemcpyAsync(b.ksig.p, ksig.data(), 4 * n, hipMemcpyHostToDevice, d.stream));
    NWV_HIP(hipStreamSynchronize(d.stream));
    b.nkeys_distinct = m;
    return NWV_OK;
}

bool verdicts_all_valid(const uint64_t* bits, size_t n) {''')
s = s.replace('''// in the range are renumbered densely, uploaded with the CSR of signatures per key, and pk is
// expanded per signature (the per-signature fallback reads it).  Call after ed_stage with
// pk == nullptr... i.e. ed_stage_keyed does both.''', '''// in the range are renumbered densely, uploaded with the CSR of signatures per key, and pk is
// expanded per signature (the per-signature fallback reads it).''')
# ed_stage must clear the keyed state (a plain staging after a keyed one)
rep('''    NWV_HIP(hipStreamSynchronize(d.stream));  // `off` is a host temporary
    return NWV_OK;
}''', '''    NWV_HIP(hipStreamSynchronize(d.stream));  // `off` is a host temporary
    b.nkeys_distinct = 0;
    return NWV_OK;
}''')
open(p, 'w').write(s)
print('host patched')
