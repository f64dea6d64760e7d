"""CPU checks of the GPU tests' closeness criterion (tests/numerics.py): it accepts an output
that is the oracle rounded to the kernel's dtype, and rejects errors a max-normalised bound
(``max|a - b| <= tol * max|b|``, the round-2 check) let through."""
import pytest
import torch

from numerics import check_close, check_elem, close_ratio

DT = [torch.bfloat16, torch.float16]
# the largest k any GPU kernel test may use (tests/test_kernels_gpu.py asserts its k's stay below)
K_MAX = {torch.bfloat16: 5.0, torch.float16: 5.0}


@pytest.mark.parametrize("dt", DT)
def test_rounded_oracle_passes(dt):
    g = torch.Generator().manual_seed(0)
    ref = torch.randn(64, 512, generator=g, dtype=torch.float64)
    assert close_ratio(ref.to(dt), ref, dt) <= 1.0 + 1e-9
    check_close(ref.to(dt), ref, dt, k=1.0)


@pytest.mark.parametrize("dt", DT)
def test_rejects_small_magnitude_perturbation(dt):
    """1 % (of the RMS) added to the smallest-magnitude 10 % of elements only."""
    g = torch.Generator().manual_seed(1)
    ref = torch.randn(128, 256, generator=g, dtype=torch.float64)
    out = ref.to(dt).double()
    small = ref.abs().flatten().argsort()[: ref.numel() // 10]
    rms = ref.pow(2).mean().sqrt()
    out.view(-1)[small] += 0.01 * rms
    # the round-2 bound (bf16: 2e-2 x max|ref|, x4 for attention backward) does not see it
    assert (out - ref).abs().max() <= 2e-2 * ref.abs().max()
    # the new one does, even at the loosest k the kernel tests use for this dtype (K_MAX)
    assert close_ratio(out, ref, dt) > K_MAX[dt]
    with pytest.raises(AssertionError):
        check_close(out, ref, dt, k=K_MAX[dt])


@pytest.mark.parametrize("dt", DT)
def test_rejects_one_wrong_row(dt):
    """One of 256 rows (a masked-tile edge / a wrong GQA partial) off by 5 %."""
    g = torch.Generator().manual_seed(2)
    ref = torch.randn(256, 128, generator=g, dtype=torch.float64)
    out = ref.to(dt).double()
    out[17] *= 1.05
    assert close_ratio(out, ref, dt) > 2.0
    with pytest.raises(AssertionError):
        check_close(out, ref, dt, k=2.0)


def test_rejects_nan_and_passes_fp32_summation_noise():
    ref = torch.randn(1000, dtype=torch.float64)
    bad = ref.clone()
    bad[3] = float("nan")
    with pytest.raises(AssertionError):
        check_close(bad, ref, torch.float32)
    check_close(ref.float() * (1 + 1e-7), ref, torch.float32, k=1.0)


def test_elementwise_check():
    ref = torch.linspace(1, 10, 100, dtype=torch.float64)
    check_elem(ref * (1 + 1e-6), ref, rtol=2e-6, atol=0)
    bad = ref.clone()
    bad[50] += 1e-3
    with pytest.raises(AssertionError):
        check_elem(bad, ref, rtol=1e-5, atol=1e-5)
