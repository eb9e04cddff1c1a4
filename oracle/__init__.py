"""CPU oracle for the argus training hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
anything from this package, and only as the *checker* (or the timed CPU baseline). The product
package ``argus_amd`` never imports it; its GPU path fails loudly when the HIP library is missing.

Contents
--------
- ``oracle.resnet``  : torchvision ResNet-50 v1.5 restated in plain ``torch.nn`` (same module names,
                       construction order and init rules, so seeded weights and ``state_dict`` keys
                       match the reference's ``models.resnet50`` call at ``argus/models.py:43``).
- ``oracle.ncamera`` : ``NCameraCNN`` / ``NCameraCNNConfig`` restated from ``argus/models.py:13-90``.
- ``oracle.se3``     : the pypose SE(3) arithmetic behind ``geometric_loss_fn``
                       (``argus/train.py:105-119``) restated in closed form (fp64-capable).
- ``oracle.step``    : the reference train step (``argus/train.py:298-321``) on CPU.

Pinning: ``tests/golden/make_golden.py`` executes the reference's own
``argus/models.py`` source (in the build container only) against ``oracle.resnet`` injected as
``torchvision.models`` and checks the two NCameraCNNs agree bit-for-bit; the SE(3) loss is pinned
by the reference's identity test (``tests/test_train.py:32-36``) and closed-form known answers.
torchvision's and pypose's own arithmetic is not in ``/root/reference`` (unpinned third-party
dependencies, ``pyproject.toml:24,27``) — it is restated from their published definitions.
"""
