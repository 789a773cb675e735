// rt_libm.h — sin and cos exactly as the reference's runtime computes them.
//
// The reference's flonum sin / cos are the C library's (Gauche calls libm),
// and so are the oracle's (oracle/rt_oracle.c, built -fno-builtin).  OCML's
// sin / cos (the device library) are within 1 ulp but not the same function:
// a 1-ulp change of a lambertian bounce direction (random-cosine-direction,
// util.scm:37-44, Q29) is enough to change which curve a grazing ray hits in
// a dense ribbon cloud, so curve scenes drifted from the oracle pixel by
// pixel.  Here sin / cos restate the platform libm's algorithm so the device
// computes the same bits: glibc 2.35 sysdeps/ieee754/dbl-64/s_sin.c (the IBM
// Accurate Mathematical Library: argument reduction by pi/2 in four parts,
// a 1/128-spaced table of sin / cos as double-doubles, short Taylor-style
// corrections), as x86-64 glibc runs it on a CPU with FMA — its multiarch
// __sin_fma / __cos_fma, the same source compiled with -mfma, where GCC fuses
// every product whose uses are all additions into an FMA.  The fusions below
// are written out as fma() calls; nothing else may be contracted
// (-ffp-contract=off).  The table holds round-to-nearest sin(k/128), cos(k/128)
// and the rounded remainders.
//
// Checked on the host against the C library bit for bit
// (tests/csrc/libm_check.cpp, tests/test_libm.py: 0 differences over 2e7
// random arguments, the random-cosine-direction angles 2 pi u included).
// sin_ / cos_ are valid for |x| < 0x1.921fbp+26, the reference algorithm's fast
// reduction range (beyond it glibc switches to a Payne-Hanek reduction this
// file does not restate); sin_full / cos_full / sincos_full take every
// argument and fall back to the platform's function outside that range (the
// bounce angles lie in (0, 2 pi), but marble's sin(scale z + 10 turb) follows
// the scene's scale).  The table may be passed in: the shade kernels stage a
// copy in LDS (rt_kernels.hip).
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#ifdef __HIPCC__
#define RT_LIBM_FN __device__ __forceinline__
#define RT_LIBM_TAB __device__ __constant__
#else
#define RT_LIBM_FN static inline
#define RT_LIBM_TAB static const
#endif

namespace rtlibm {

RT_LIBM_TAB double kSinCosTab[4 * 112] = {   // sin(k/128) hi, lo, cos(k/128) hi, lo
    0x0.0p+0, 0x0.0p+0, 0x1.0000000000000p+0, 0x0.0p+0,   /* k = 0 */
    0x1.fffeaaaaeeeefp-8, -0x1.e45e2ec67b77cp-62, 0x1.fffc000155552p-1, 0x1.f4a01a0196daep-55,   /* k = 1 */
    0x1.fffaaaaeeeed5p-7, -0x1.2ab639a9f0776p-63, 0x1.fff000155549fp-1, 0x1.28a28a03a5ef3p-55,   /* k = 2 */
    0x1.7ff7001033255p-6, 0x1.efe2b51527336p-64, 0x1.ffdc006bff7e6p-1, 0x1.ae6dae86977bdp-55,   /* k = 3 */
    0x1.ffeaaaeeee86fp-6, -0x1.cd406fb224ae2p-60, 0x1.ffc00155527d3p-1, -0x1.3b54492d89b5bp-55,   /* k = 4 */
    0x1.3feb2b12d45d5p-5, 0x1.4ec54203d1c11p-60, 0x1.ff9c03414a7bap-1, 0x1.991f4be6c59bfp-57,   /* k = 5 */
    0x1.7fdc01032fba9p-5, -0x1.599bdf46e997ap-59, 0x1.ff7006bfdf99fp-1, -0x1.8b3b560648d5fp-56,   /* k = 6 */
    0x1.bfc6d78586dacp-5, 0x1.8e4fd03dbf236p-62, 0x1.ff3c0c8103a31p-1, 0x1.4856dbddc0e66p-56,   /* k = 7 */
    0x1.ffaaaeeed4edbp-5, -0x1.2d16d32684b69p-59, 0x1.ff0015549f4d3p-1, 0x1.328387b99426fp-55,   /* k = 8 */
    0x1.1fc343d808befp-4, -0x1.f3d32e6f3be4fp-58, 0x1.febc222a8ef9fp-1, 0x1.7934934f54c77p-58,   /* k = 9 */
    0x1.3facb12d1755bp-4, -0x1.921915299468bp-58, 0x1.fe7034129ef6fp-1, -0x1.cbf4337c96f97p-57,   /* k = 10 */
    0x1.5f911fd10b737p-4, -0x1.0184f02be9102p-58, 0x1.fe1c4c3c873ebp-1, -0x1.5a9c9057c4a02p-60,   /* k = 11 */
    0x1.7f701032550e4p-4, 0x1.afc2d1800501ap-60, 0x1.fdc06bf7e6b9bp-1, 0x1.31902b535f8dbp-55,   /* k = 12 */
    0x1.9f4902d55d1f9p-4, 0x1.2696d7eac1dc1p-58, 0x1.fd5c94b43e000p-1, -0x1.2e768cb4f92f9p-57,   /* k = 13 */
    0x1.bf1b78568391dp-4, 0x1.e91841dea4cc8p-58, 0x1.fcf0c800e99b1p-1, 0x1.ea3d786d186acp-57,   /* k = 14 */
    0x1.dee6f16c1cce6p-4, -0x1.50f8e2fb71673p-59, 0x1.fc7d078d1bc88p-1, 0x1.075d2447db685p-55,   /* k = 15 */
    0x1.feaaeee86ee36p-4, -0x1.afcb2bcc6f03bp-59, 0x1.fc015527d5bd3p-1, 0x1.b68f35094efb8p-55,   /* k = 16 */
    0x1.0f3378ddd71d1p-3, 0x1.d8468724f0f9ep-57, 0x1.fb7db2bfe0695p-1, 0x1.21dadf4f65ab1p-55,   /* k = 17 */
    0x1.1f0d3d7afceafp-3, -0x1.6ef95099769a5p-57, 0x1.faf22263c4bd3p-1, -0x1.52ace133a2769p-58,   /* k = 18 */
    0x1.2ee285e4ab88fp-3, -0x1.e4d0f05dee058p-57, 0x1.fa5ea641c36f2p-1, 0x1.04da6ed17cc7cp-59,   /* k = 19 */
    0x1.3eb312c5d66cbp-3, 0x1.47d666b66cb91p-57, 0x1.f9c340a7cc428p-1, 0x1.c5b6b063b7462p-55,   /* k = 20 */
    0x1.4e7ea4dc5f27bp-3, 0x1.949db2ac072fcp-58, 0x1.f91ff40374d01p-1, -0x1.7d03f4d3a9e4cp-57,   /* k = 21 */
    0x1.5e44fcfa126f3p-3, -0x1.6f443063f89b6p-57, 0x1.f874c2e1eecf6p-1, -0x1.c6514e1332b16p-55,   /* k = 22 */
    0x1.6e05dc05a4d4cp-3, -0x1.32c5c8b81c919p-66, 0x1.f7c1afeffde24p-1, -0x1.8f55bc47540b1p-56,   /* k = 23 */
    0x1.7dc102fbaf2b5p-3, 0x1.5ab50e23c97c3p-59, 0x1.f706bdf9ece1cp-1, -0x1.698c80c36dcb4p-55,   /* k = 24 */
    0x1.8d7632efaa944p-3, -0x1.20fa262cbb953p-57, 0x1.f643efeb82acdp-1, 0x1.6b00ac1fe28acp-56,   /* k = 25 */
    0x1.9d252d0cec312p-3, 0x1.9c43d80b1137dp-58, 0x1.f57948cff6797p-1, 0x1.e3a0d3e03b1d4p-57,   /* k = 26 */
    0x1.accdb297a0765p-3, -0x1.9883b57d6cdeap-58, 0x1.f4a6cbd1e3a79p-1, 0x1.13df0edaebb57p-55,   /* k = 27 */
    0x1.bc6f84edc6199p-3, 0x1.9c1a56a7b0cabp-57, 0x1.f3cc7c3b3d16ep-1, -0x1.21a3ad28a3494p-57,   /* k = 28 */
    0x1.cc0a6588289a3p-3, -0x1.868d09bc87c6bp-57, 0x1.f2ea5d753ffedp-1, 0x1.cc4215f56d583p-55,   /* k = 29 */
    0x1.db9e15fb5a5d0p-3, -0x1.32e20d6cc6fc2p-57, 0x1.f20073086649fp-1, 0x1.b940416c1984bp-56,   /* k = 30 */
    0x1.eb2a57f8ae5a3p-3, -0x1.0be06af572cebp-57, 0x1.f10ec09c5873bp-1, 0x1.d9072762c1283p-55,   /* k = 31 */
    0x1.faaeed4f31577p-3, -0x1.15d88508e32b8p-57, 0x1.f01549f7deea1p-1, 0x1.d3c1e99e5cafdp-55,   /* k = 32 */
    0x1.0515cbf65155cp-2, -0x1.9b8c29dfd8ec7p-56, 0x1.ef141300d2f26p-1, -0x1.2aa1b08ded372p-55,   /* k = 33 */
    0x1.0cd00cef36436p-2, -0x1.9fb0a0c93e2b4p-56, 0x1.ee0b1fbc0f11cp-1, -0x1.bfd2380bbc3b1p-59,   /* k = 34 */
    0x1.14861aa94ddebp-2, -0x1.be881b5b615a4p-57, 0x1.ecfa744d5efa1p-1, -0x1.56d0a4af541d0p-58,   /* k = 35 */
    0x1.1c37d64c6b876p-2, 0x1.46076fe0dcff4p-56, 0x1.ebe214f76efa8p-1, -0x1.02f9f12ba543ep-55,   /* k = 36 */
    0x1.23e52111aaf36p-2, -0x1.4f080334eff18p-56, 0x1.eac2061bbaf4fp-1, 0x1.2c1d53e94658dp-57,   /* k = 37 */
    0x1.2b8ddc43eb49fp-2, 0x1.1553899f2d807p-57, 0x1.e99a4c3a7cd83p-1, -0x1.2264b1bc53ce8p-55,   /* k = 38 */
    0x1.3331e94049f87p-2, 0x1.e0cb6b40c302cp-56, 0x1.e86aebf29a9edp-1, 0x1.9397afdbb58a7p-55,   /* k = 39 */
    0x1.3ad129769d3d8p-2, 0x1.03d550487839ap-63, 0x1.e733ea0193d40p-1, -0x1.6428b3546ce13p-55,   /* k = 40 */
    0x1.426b7e69ee697p-2, -0x1.f09c75705c59fp-56, 0x1.e5f54b436e9d0p-1, 0x1.7eb0fd02fc8bcp-55,   /* k = 41 */
    0x1.4a00c9b0f3d20p-2, 0x1.823ba6bb08eadp-56, 0x1.e4af14b2a449cp-1, -0x1.68ca02e8a6833p-55,   /* k = 42 */
    0x1.5190ecf68a77ap-2, 0x1.b357155eef0f3p-56, 0x1.e3614b680d6a5p-1, -0x1.27793aa015237p-56,   /* k = 43 */
    0x1.591bc9fa2f597p-2, 0x1.7c74bac3fe0cbp-57, 0x1.e20bf49acd6c1p-1, -0x1.660aec7ef636bp-58,   /* k = 44 */
    0x1.60a1429078775p-2, 0x1.b1fd80ba89133p-58, 0x1.e0af15a03dbcep-1, 0x1.fe8e702771ae6p-58,   /* k = 45 */
    0x1.682138a38d7f7p-2, -0x1.d889202444aadp-56, 0x1.df4ab3ebd875ep-1, -0x1.e2d8a7e6736c4p-55,   /* k = 46 */
    0x1.6f9b8e33a0255p-2, 0x1.42bc14ee9da0dp-56, 0x1.ddded50f228d6p-1, -0x1.e80c8d42ba2bfp-57,   /* k = 47 */
    0x1.7710255764214p-2, -0x1.6ead7314bb6cep-57, 0x1.dc6b7eb995912p-1, 0x1.4b364776dcd35p-58,   /* k = 48 */
    0x1.7e7ee03c86d4ep-2, -0x1.b63bcdabf5af2p-56, 0x1.daf0b6b888e83p-1, 0x1.a249e2b5e5ceap-55,   /* k = 49 */
    0x1.85e7a12826949p-2, 0x1.8a40e9b5face0p-56, 0x1.d96e82f71a9dcp-1, 0x1.ff61bd5d2039dp-55,   /* k = 50 */
    0x1.8d4a4a774992fp-2, 0x1.44a02ea766326p-56, 0x1.d7e4e97e17b4ap-1, -0x1.3b770352bed94p-57,   /* k = 51 */
    0x1.94a6be9f546c5p-2, -0x1.69ce13e683f58p-56, 0x1.d653f073e4040p-1, -0x1.76236434bec37p-55,   /* k = 52 */
    0x1.9bfce02e80510p-2, 0x1.09e39a320b0a4p-56, 0x1.d4bb9e1c619e0p-1, 0x1.f34bb77858f61p-55,   /* k = 53 */
    0x1.a34c91cc50ccap-2, -0x1.a310e3b50cecdp-58, 0x1.d31bf8d8d7c06p-1, 0x1.e60dd3089cbddp-56,   /* k = 54 */
    0x1.aa95b63a09277p-2, -0x1.6293eb13c0381p-57, 0x1.d1750727d94f0p-1, 0x1.0d52b1ec1a48ep-55,   /* k = 55 */
    0x1.b1d8305321617p-2, -0x1.ae242cb99f519p-56, 0x1.cfc6cfa52ad9fp-1, 0x1.8b5b5508f2a0dp-55,   /* k = 56 */
    0x1.b913e30dbac43p-2, -0x1.e38ad2f6c3ff1p-56, 0x1.ce115909a82e5p-1, 0x1.1f139bb31109ap-55,   /* k = 57 */
    0x1.c048b17b140a3p-2, 0x1.19fe6757e9fa7p-57, 0x1.cc54aa2b2972ep-1, 0x1.4ee162ba83a98p-57,   /* k = 58 */
    0x1.c7767ec7fd19ep-2, -0x1.eb14d1a3d5826p-58, 0x1.ca90c9fc67d0bp-1, -0x1.46a81485e3462p-57,   /* k = 59 */
    0x1.ce9d2e3d4a51fp-2, -0x1.2fc8a12dae298p-57, 0x1.c8c5bf8ce1a84p-1, 0x1.ab3d1a1590123p-56,   /* k = 60 */
    0x1.d5bca34047661p-2, 0x1.28a44a75fc29cp-56, 0x1.c6f39208be53bp-1, -0x1.741dbfbaadb42p-55,   /* k = 61 */
    0x1.dcd4c15329c9ap-2, 0x1.0d4c6e171fd9ap-56, 0x1.c51a48b8b175ep-1, -0x1.1bbb43b9aa880p-57,   /* k = 62 */
    0x1.e3e56c1582a69p-2, -0x1.0a4821099f88fp-58, 0x1.c339eb01ddd81p-1, -0x1.caaf5ee82c5c0p-55,   /* k = 63 */
    0x1.eaee8744b05f0p-2, -0x1.789b43c9b027dp-58, 0x1.c1528065b7d50p-1, -0x1.892111312e828p-55,   /* k = 64 */
    0x1.f1eff6bc4f97bp-2, 0x1.17212f8a7525cp-56, 0x1.bf641081e7536p-1, 0x1.b7bd71628a9a1p-55,   /* k = 65 */
    0x1.f8e99e76abc97p-2, 0x1.9d950af2d00a3p-58, 0x1.bd6ea310294f5p-1, 0x1.31bbcc88c109dp-56,   /* k = 66 */
    0x1.ffdb628d2f57ap-2, 0x1.f4a992e905b6ap-57, 0x1.bb723fe630f32p-1, 0x1.72bd2452d0a39p-56,   /* k = 67 */
    0x1.0362939c69955p-1, -0x1.2d8cd78397b01p-55, 0x1.b96eeef58840ep-1, 0x1.45a3cc78fade0p-58,   /* k = 68 */
    0x1.06d3686946e5bp-1, 0x1.3f5ae4538ff1bp-55, 0x1.b764b84b704c2p-1, -0x1.f5848c21b389bp-55,   /* k = 69 */
    0x1.0a4021e9e1001p-1, -0x1.6f643a13914f6p-55, 0x1.b553a410c104ep-1, 0x1.8ff7947027a15p-58,   /* k = 70 */
    0x1.0da8b26b5672ep-1, -0x1.a58def0bee909p-55, 0x1.b33bba89c8948p-1, 0x1.ea6a51d1f6ca9p-55,   /* k = 71 */
    0x1.110d0c4b69c3bp-1, 0x1.d918998809981p-55, 0x1.b11d04162a4c6p-1, 0x1.1dd561efbc0c2p-56,   /* k = 72 */
    0x1.146d21f8b7f82p-1, 0x1.bf9535e2739a8p-56, 0x1.aef78930bd275p-1, -0x1.f836279746f94p-56,   /* k = 73 */
    0x1.17c8e5f2eedb0p-1, 0x1.35e57102e2488p-57, 0x1.accb526f69de5p-1, 0x1.8fb6a8dd6b6ccp-55,   /* k = 74 */
    0x1.1b204acb02fddp-1, -0x1.f190c70cbb5fep-58, 0x1.aa98688308913p-1, -0x1.b83d607cd5072p-63,   /* k = 75 */
    0x1.1e7343236574cp-1, 0x1.22a3fa4f41d5ap-56, 0x1.a85ed4373e02dp-1, 0x1.9be06385ec792p-57,   /* k = 76 */
    0x1.21c1c1b0394cfp-1, 0x1.e5b324b23aa31p-58, 0x1.a61e9e72586afp-1, 0x1.58330e2fd453fp-55,   /* k = 77 */
    0x1.250bb93788bbbp-1, 0x1.ea3d02457bccep-56, 0x1.a3d7d0352bdcfp-1, -0x1.68dbaeca19669p-55,   /* k = 78 */
    0x1.28511c917a067p-1, -0x1.01df1d9a16b70p-55, 0x1.a18a729aee445p-1, 0x1.95e25736c0357p-60,   /* k = 79 */
    0x1.2b91dea88421ep-1, -0x1.fa371db216ab0p-55, 0x1.9f368ed912f85p-1, -0x1.1d200c5791606p-55,   /* k = 80 */
    0x1.2ecdf279a3082p-1, 0x1.d3557e0e7e37ep-55, 0x1.9cdc2e3f25e5cp-1, 0x1.3f99112993f62p-55,   /* k = 81 */
    0x1.32054b148bc4fp-1, 0x1.f6b42095a135bp-55, 0x1.9a7b5a36a6514p-1, 0x1.722cfcc9fa7a9p-55,   /* k = 82 */
    0x1.3537db9be0367p-1, 0x1.b327e7af040f0p-57, 0x1.98141c42e1310p-1, 0x1.d1ff80488f08dp-55,   /* k = 83 */
    0x1.386597456282bp-1, -0x1.10fada93b07a8p-56, 0x1.95a67e00cb1fdp-1, -0x1.0befda21f862dp-55,   /* k = 84 */
    0x1.3b8e715a2840ap-1, -0x1.97653a7d2f07ap-56, 0x1.93328926d9e92p-1, -0x1.bb77003600cdap-55,   /* k = 85 */
    0x1.3eb25d36cd53ap-1, -0x1.be570e1570fc0p-58, 0x1.90b84784ddaf7p-1, -0x1.0feb10ab93b87p-56,   /* k = 86 */
    0x1.41d14e4ba6790p-1, 0x1.4608fd287ecf5p-55, 0x1.8e37c303d9ad1p-1, -0x1.463a4b53d4bf8p-57,   /* k = 87 */
    0x1.44eb381cf386bp-1, -0x1.3ed6c1e6a5505p-55, 0x1.8bb105a5dc900p-1, 0x1.863e03e9474c1p-55,   /* k = 88 */
    0x1.48000e431159fp-1, -0x1.b194a7463ed10p-55, 0x1.89241985d871fp-1, 0x1.c48d9c413ed84p-55,   /* k = 89 */
    0x1.4b0fc46aab761p-1, 0x1.0da05738cc59cp-61, 0x1.869108d77a6c6p-1, 0x1.338ffe2bfe9ddp-56,   /* k = 90 */
    0x1.4e1a4e54ed51bp-1, -0x1.a492f89b7c76ap-55, 0x1.83f7dde701ca0p-1, -0x1.152cf609bc6e8p-59,   /* k = 91 */
    0x1.511f9fd7b351cp-1, -0x1.5c0e861c48831p-55, 0x1.8158a31916d5dp-1, -0x1.de8b90b8228dep-57,   /* k = 92 */
    0x1.541facddbb724p-1, 0x1.232c28520d391p-56, 0x1.7eb362eaa1488p-1, 0x1.a1d65a4a5959fp-58,   /* k = 93 */
    0x1.571a6966d59b3p-1, 0x1.c843b4d0fb197p-58, 0x1.7c0827f09e54fp-1, -0x1.c73d6d72aee68p-57,   /* k = 94 */
    0x1.5a0fc98813a12p-1, -0x1.d82e2b7d4227bp-55, 0x1.7956fcd7f6543p-1, -0x1.ab276e9d45ae4p-55,   /* k = 95 */
    0x1.5cffc16bf8f0dp-1, 0x1.96cb370eb578ap-55, 0x1.769fec655211fp-1, -0x1.827d5cf8c68c5p-57,   /* k = 96 */
    0x1.5fea4552a9e57p-1, 0x1.0b6cef7ee20b7p-55, 0x1.73e30174efba1p-1, -0x1.5d3ae3d94ad5fp-57,   /* k = 97 */
    0x1.62cf49921ac79p-1, -0x1.edd9855b6241ap-55, 0x1.712046fa77678p-1, 0x1.425b0a5029c81p-55,   /* k = 98 */
    0x1.65aec2963e755p-1, 0x1.126f96b71053cp-55, 0x1.6e57c800cf55ep-1, 0x1.60286dedbd0a6p-55,   /* k = 99 */
    0x1.6888a4e134b2fp-1, -0x1.6b7d37644d5e6p-55, 0x1.6b898fa9efb5dp-1, 0x1.15ac786ccf4b2p-56,   /* k = 100 */
    0x1.6b5ce50b7821ap-1, -0x1.5d5158f702e0fp-57, 0x1.68b5a92eb6253p-1, -0x1.9a91ad985f89cp-55,   /* k = 101 */
    0x1.6e2b77c40bde1p-1, -0x1.0e729857fad53p-56, 0x1.65dc1fdeb8cbap-1, -0x1.97c1b47337c77p-58,   /* k = 102 */
    0x1.70f451d0a8c40p-1, 0x1.97ede3885770dp-57, 0x1.62fcff20191c7p-1, 0x1.d9143895756efp-57,   /* k = 103 */
    0x1.73b7680dea578p-1, -0x1.2248306dc12a2p-56, 0x1.6018526f563dfp-1, 0x1.46ca5e0e432d0p-55,   /* k = 104 */
    0x1.7674af6f7b524p-1, 0x1.e9d3f94ac84a8p-56, 0x1.5d2e255f1f17ap-1, 0x1.0314104c8892bp-55,   /* k = 105 */
    0x1.792c1d0041d52p-1, -0x1.abf05eeb354ebp-55, 0x1.5a3e839824077p-1, 0x1.428aa2759be62p-55,   /* k = 106 */
    0x1.7bdda5e28b3c2p-1, 0x1.ad1197ccd0392p-59, 0x1.574978d8e83f2p-1, 0x1.f4714af282d23p-55,   /* k = 107 */
    0x1.7e893f5037959p-1, 0x1.0eefbaa650c4cp-55, 0x1.544f10f592ca5p-1, -0x1.e7ae8e6c7a62fp-55,   /* k = 108 */
    0x1.812ede9ae4ba4p-1, -0x1.7830adf402ddap-55, 0x1.514f57d7bf3dap-1, 0x1.47a108073c259p-56,   /* k = 109 */
    0x1.83ce792c1906ep-1, -0x1.f3899682b4a7dp-56, 0x1.4e4a597e4e10ep-1, 0x1.ccd992849f6c8p-56,   /* k = 110 */
    0x1.866804856db62p-1, 0x1.407b4e7476623p-57, 0x1.4b4021fd34a33p-1, -0x1.ee903cecc18cbp-55,   /* k = 111 */
};

RT_LIBM_FN uint64_t bits(const double x) {
#ifdef __HIPCC__
    return (uint64_t)__double_as_longlong(x);
#else
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
#endif
}

constexpr double kBig = 52776558133248.0;                       // 0x1.8p45: big + |x| rounds |x| to k/128
constexpr double kSn3 = -1.66666666666664880952546298448555E-01, kSn5 = 8.33333214285722277379541354343671E-03;
constexpr double kCs2 = 4.99999999999999999999950396842453E-01, kCs4 = -4.16666666666664434524222570944589E-02;
constexpr double kCs6 = 1.38888874007937613028114285595617E-03;
constexpr double kS1 = -0x1.5555555555555p-3, kS2 = 0x1.1111111110ECEp-7, kS3 = -1.9841269834414642e-04;
constexpr double kS4 = 2.755729806860771e-06, kS5 = -2.5022014848318398e-08;
constexpr double kHp0 = 0x1.921fb54442d18p+0, kHp1 = 0x1.1a62633145c07p-54;   // pi/2 as a double-double
constexpr double kHpInv = 0x1.45f306dc9c883p-1, kToInt = 6755399441055744.0;
constexpr double kMp1 = 0x1.921FB58000000p0, kMp2 = -0x1.DDE973C000000p-27;    // pi/2 in four parts
constexpr double kPp3 = -0x1.CB3B398000000p-55, kPp4 = -0x1.d747f23e32ed7p-83;

// One evaluation of the reference algorithm's kernels on a reduced argument
// a + da: do_cos (cq) or do_sin (!cq), including do_sin's short series for
// |a| < 0.126.  The kernels differ only in a few operations, so they are one
// straight-line evaluation with selects (no divergent branches under SIMT, and
// one set of temporaries).  In the reference: do_cos first flips da with the
// sign of a and adds it to the table offset; do_sin flips it when a <= 0 and
// carries it separately.
RT_LIBM_FN double core(const double a, double da, const bool cq, const double* tab) {
    // do_sin, |a| < 0.126: a - a^3/3! + ... + (1 - a^2) da / 2
    const double aa = a * a;
    const double poly = fma(fma(fma(fma(kS5, aa, kS4), aa, kS3), aa, kS2), aa, kS1);
    const double taylor = a + fma(fma(poly, a, -(0.5 * da)), aa, da);
    // the table kernels
    if (cq ? (a < 0) : (a <= 0)) da = -da;
    const double u = kBig + fabs(a);
    const double x0 = fabs(a) - (u - kBig);
    const double x = cq ? x0 + da : x0;
    const double d = cq ? 0.0 : da;
    const double xx = x * x;
    const double m = x * xx, ps = fma(xx, kSn5, kSn3);
    const double s = cq ? fma(m, ps, x) : x + fma(m, ps, d);
    const double c = fma(x, d, xx * fma(xx, fma(xx, kCs6, kCs4), kCs2));
    uint32_t k = (uint32_t)bits(u);
    k = (k < 112u ? k : 111u) << 2;
    const double sn = tab[k], ssn = tab[k + 1], cs = tab[k + 2], ccs = tab[k + 3];
    // do_cos: cor = (ccs - s ssn - cs c) - sn s, result cs + cor;
    // do_sin: cor = (ssn + s ccs - sn c) + cs s, result sn + cor with a's sign
    const double w3 = cq ? -ssn : ccs, w4 = cq ? ccs : ssn, w2 = cq ? -cs : -sn, w1 = cq ? -sn : cs;
    const double cor = fma(w1, s, fma(w2, c, fma(s, w3, w4)));
    const double r = (cq ? cs : sn) + cor;
    const double table = cq ? r : copysign(r, a);
    return (!cq && fabs(a) < 0.126) ? taylor : table;
}
// x = n (pi/2) + (a + da), |a| <= pi/4; returns n mod 4
RT_LIBM_FN int reduce_sincos(const double x, double& a, double& da) {
    const double t = fma(x, kHpInv, kToInt);
    const double xn = t - kToInt;
    const double y = fma(-xn, kMp2, fma(-xn, kMp1, x));
    const int n = (int)((uint32_t)bits(t) & 3u);
    const double t2 = fma(-xn, kPp3, y);
    double db = fma(-xn, kPp3, y - t2);
    const double b = fma(-xn, kPp4, t2);
    db += fma(-xn, kPp4, t2 - b);
    a = b;
    da = db;
    return n;
}
// high word without the sign: the reference algorithm's range dispatch
RT_LIBM_FN uint32_t hiword(const double x) { return (uint32_t)(bits(x) >> 32) & 0x7fffffffu; }

RT_LIBM_FN bool in_range(const double x) { return hiword(x) < 0x419921FBu; }

// sin (cos_ = false) or cos (true) of x, |x| < 0x1.921fbp+26 (in_range).  The
// reference's range cases — |x| < 0.855469: the kernel on x itself; up to
// 2.426265: the other kernel on pi/2 - |x| (as a double-double); beyond: the
// kernel picked by the quadrant of the four-part reduction — all come down to
// one core() call on (a, da) and a sign.
RT_LIBM_FN double sincos_(const double x, const bool want_cos, const double* tab = kSinCosTab) {
    const uint32_t hw = hiword(x);
    double a = x, da = 0.0, sign = 1.0;
    bool cq = want_cos;
    if (hw >= 0x400368fdu) {                                    // 2.426265 <= |x|
        double ra, rda;
        const int n = reduce_sincos(x, ra, rda) + (want_cos ? 1 : 0);
        a = ra; da = rda;
        cq = (n & 1) != 0;
        sign = (n & 2) ? -1.0 : 1.0;
    } else if (hw >= 0x3feb6000u) {                             // 0.855469 <= |x| < 2.426265
        const double y = kHp0 - fabs(x);
        if (want_cos) {                                         // do_sin(y + hp1 as a double-double)
            a = y + kHp1;
            da = (y - a) + kHp1;
            cq = false;
        } else {                                                // copysign(do_cos(y, hp1), x)
            a = y;
            da = kHp1;
            cq = true;
            sign = copysign(1.0, x);
        }
    }
    const double r = core(a, da, cq, tab);
    const double tiny = want_cos ? 1.0 : x;                     // |x| < 2^-27 (cos) / 2^-26 (sin)
    const bool is_tiny = hw < (want_cos ? 0x3e400000u : 0x3e500000u);
    return is_tiny ? tiny : (sign < 0.0 ? -r : r);
}
RT_LIBM_FN double sin_(const double x) { return sincos_(x, false); }
RT_LIBM_FN double cos_(const double x) { return sincos_(x, true); }

// Every argument: the restatement inside its reduction range; beyond it (|x| >= 0x1.921fbp+26, where the
// reference algorithm switches to its Payne-Hanek reduction, and inf / nan) the platform's own function
// — the device library on the GPU (within 1 ulp), the C library itself on the host.
RT_LIBM_FN double sincos_full(const double x, const bool want_cos, const double* tab = kSinCosTab) {
    if (in_range(x)) return sincos_(x, want_cos, tab);
    return want_cos ? ::cos(x) : ::sin(x);
}
RT_LIBM_FN double sin_full(const double x) { return sincos_full(x, false); }
RT_LIBM_FN double cos_full(const double x) { return sincos_full(x, true); }

}  // namespace rtlibm
