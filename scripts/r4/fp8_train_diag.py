"""Round-4 diagnosis of tests/test_fp8_inference.py::test_fp8_value_training_tracks_bf16[152-False-False]
(fp8 forward + bf16 backward: the loss on 32 memorised boards went UP over 15 steps).  Prints the
per-step loss of the bf16 trainer and of the fp8 trainer in each (fp8_dgrad, fp8_wgrad) arm, with the
fused update on and off.  Usage: python scripts/r4/fp8_train_diag.py"""
import copy
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402


def main():
    from alphago_amd.models.nets import ValueNet
    from alphago_amd.train.engine import HipValueTrainer

    dev = torch.device("cuda")
    torch.manual_seed(0)
    B = 32
    net0 = ValueNet(49, filters_per_layer=152, layers=4)
    g = torch.Generator().manual_seed(5)
    planes = torch.randint(0, 2, (B, 49, 19, 19), dtype=torch.uint8, generator=g).to(dev)
    z = (torch.randint(0, 2, (B,), device=dev) * 2 - 1).float()
    arms = [("bf16", None, None, "1"), ("fp8", False, False, "1"), ("fp8", False, False, "0"),
            ("fp8", True, True, "1"), ("fp8", True, False, "1"), ("fp8", False, True, "1")]
    for prec, dg, wg, fused in arms:
        os.environ["ALPHAGO_AMD_FUSED_UPDATE"] = fused
        kw = {} if prec == "bf16" else dict(fp8_dgrad=dg, fp8_wgrad=wg)
        t = HipValueTrainer(copy.deepcopy(net0), B, lr=0.05, device=dev, precision=prec, **kw)
        losses = [round(t.evaluate(planes, z)[0].item(), 3)]
        for _ in range(15):
            t.step(planes, z)
            losses.append(round(t.evaluate(planes, z)[0].item(), 3))
        print(json.dumps({"precision": prec, "fp8_dgrad": dg, "fp8_wgrad": wg, "fused": fused, "loss": losses}),
              flush=True)


if __name__ == "__main__":
    main()
