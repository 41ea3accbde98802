"""One-off source patch (kept for the record): MSM seed in device memory + HIP-graph replay of
staged batch MSMs."""
p = '/root/repo/narwhal_amd/csrc/msm_kernels.hip'
s = open(p).read()
s = s.replace('''struct MsmSeed {
    uint32_t w[8];
};

''', '')
s = s.replace('''    const uint32_t* __restrict__ msg_len, MsmSeed seed, MsmLayout lay, uint32_t* __restrict__ ascal,''',
              '''    const uint32_t* __restrict__ msg_len, const uint32_t* __restrict__ seedp, MsmLayout lay,
    uint32_t* __restrict__ ascal,''')
s = s.replace('''        msm_z(seed.w, i, z);''', '''        uint32_t sd[8];
#pragma unroll
        for (int k = 0; k < 8; k++) sd[k] = seedp[k];
        msm_z(sd, i, z);''')
open(p, 'w').write(s)

p = '/root/repo/narwhal_amd/csrc/nwv_host.hip'
s = open(p).read()


def rep(old, new):
    global s
    assert old in s, old[:70]
    s = s.replace(old, new, 1)


# msm_launch: seed copied to m_state[8..16) (outside any graph), launches in msm_enqueue
rep('''    MsmSeed seed;
    std::memcpy(seed.w, seed32, 32);
    uint32_t* state = b.m_state.as<uint32_t>();''', '''    uint32_t* state = b.m_state.as<uint32_t>();  // [0] fail flags, [1] verdict, [8..16) seed
    if (seed32) NWV_HIP(hipMemcpyAsync(state + 8, seed32, 32, hipMemcpyHostToDevice, stream));''')
rep('''                       b.len.as<uint32_t>(), seed, p.lay, b.m_ascal.as<uint32_t>(), digits,''',
    '''                       b.len.as<uint32_t>(), state + 8, p.lay, b.m_ascal.as<uint32_t>(), digits,''')
rep('''(rc = b.m_state.ensure(64)) ||''', '''(rc = b.m_state.ensure(128)) ||''')
open(p, 'w').write(s)
print('patched')
