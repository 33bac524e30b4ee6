"""Per-call mirror of the reference surface: ``engine.Validate(PolicyContext) -> EngineResponse``
(pkg/engine/validation.go:26-140; response types pkg/engine/response/response.go:11-97), and its
batch form ``validate_batch`` (the Go side's ``ValidateBatch``), both running on
the GPU through the C ABI.

``validate`` evaluates one policy on one resource exactly as ``validateResource`` does: the
validate rules that match, in policy order, each with its ``RuleResponse`` (name, type
"Validation", message, status); ``RulesAppliedCount`` counts pass + fail and ``RulesErrorCount``
error (``addRuleResponse``, validation.go:111-123). A response without rule responses is the empty
``EngineResponse`` (``buildResponse`` returns early, validation.go:53-56). Policies are taken as
given: the CLI's defaults + autogen (``kyverno_amd.autogen``) happen before, as in the reference.

Rules the device does not evaluate (context, preconditions, deny, foreach, pattern variables other
than ``request.object`` paths: ``KV_ROUTE_CPU``) come back with status ``"cpu"``: the Go host runs
``processValidationRule`` for them. They are not counted.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from . import cli

STATUS = {0: "pass", 1: "fail", 2: "warn", 3: "error", 4: "skip", 6: "cpu"}


@dataclass
class PolicyContext:
    """pkg/engine/policyContext.go:12-45, the fields the validate path reads."""
    policy: dict
    new_resource: dict
    admission_info: dict | None = None          # kyverno.RequestInfo: roles, clusterRoles, groups, username
    exclude_group_role: list | None = None
    namespace_labels: dict | None = None        # labels of the resource's namespace (namespaceSelector)


@dataclass
class RuleResponse:
    name: str
    type: str = "Validation"
    message: str = ""
    status: str = ""


@dataclass
class ResourceSpec:
    kind: str = ""
    apiVersion: str = ""
    namespace: str = ""
    name: str = ""
    uid: str = ""


@dataclass
class PolicyResponse:
    policy_name: str = ""
    policy_namespace: str = ""
    resource: ResourceSpec = field(default_factory=ResourceSpec)
    rules_applied_count: int = 0
    rules_error_count: int = 0
    rules: list = field(default_factory=list)
    validation_failure_action: str = ""


@dataclass
class EngineResponse:
    patched_resource: dict = field(default_factory=dict)
    policy_response: PolicyResponse = field(default_factory=PolicyResponse)

    def is_successful(self) -> bool:
        """EngineResponse.IsSuccessful (response.go:115-122): no rule failed or errored."""
        return all(r.status not in ("fail", "error") for r in self.policy_response.rules)


def _response(ev: cli.Evaluation, pi: int, res: int) -> EngineResponse:
    rules = []
    for r in ev.policy_rules(pi):
        st = int(ev.status[r.index, res])
        if st == cli.NOMATCH or r.route == cli.ROUTE_NORESPONSE:
            continue
        msg = "" if st == cli.CPU else cli.rule_message(ev, r, res)
        rules.append(RuleResponse(name=r.name, message=msg, status=STATUS[st]))
    if not rules:
        return EngineResponse()
    pol, doc = ev.policies[pi], ev.resources[res]
    md, pmd = doc.get("metadata") or {}, pol.get("metadata") or {}
    return EngineResponse(
        patched_resource=doc,
        policy_response=PolicyResponse(
            policy_name=pmd.get("name", ""), policy_namespace=pmd.get("namespace", ""),
            resource=ResourceSpec(kind=doc.get("kind", ""), apiVersion=doc.get("apiVersion", ""),
                                  namespace=md.get("namespace", ""), name=md.get("name", "")),
            rules_applied_count=sum(x.status in ("pass", "fail") for x in rules),
            rules_error_count=sum(x.status == "error" for x in rules),
            rules=rules,
            validation_failure_action=(pol.get("spec") or {}).get("validationFailureAction", "")))


def validate_batch(policies: list[dict], resources: list[dict], admission_info: dict | None = None,
                   exclude_group_role: list | None = None, namespace_labels: dict | None = None, device: int = 0,
                   specialize: bool = False, gpus: int = 1) -> list[list[EngineResponse]]:
    """EngineResponse of every (policy, resource) pair, ``[policy][resource]``: one
    kv_compile + kv_ingest + kv_validate over the cross product. ``namespace_labels`` maps a
    namespace name to its labels (PolicyContext.NamespaceLabels of the resources in it)."""
    from . import batch

    ps = batch.PolicySet(policies, specialize=specialize)
    b = batch.Batch(ps, resources, namespace_labels)
    mask = ((1 << gpus) - 1) << device if gpus > 1 else None
    r = batch.validate(ps, b, admission=admission_info, exclude_group_role=exclude_group_role, device=device,
                       device_mask=mask)
    ev = cli.Evaluation(policies, resources, ps.rules, r.status)
    for ri, res in zip(*(r.status == cli.FAIL).nonzero()):
        if not ps.rules[ri].any_pattern:
            ev.paths[(int(ri), int(res))] = r.path(int(ri), int(res))
    cli.collect_errors(ev, ps, r, resources)
    cli._evaluate_anypatterns(ev, device, specialize, namespace_labels)
    return [[_response(ev, pi, res) for res in range(len(resources))] for pi in range(len(policies))]


def validate(ctx: PolicyContext, device: int = 0) -> EngineResponse:
    """engine.Validate (pkg/engine/validation.go:26) for one policy and one resource."""
    ns = (ctx.new_resource.get("metadata") or {}).get("namespace", "")
    labels = {ns: ctx.namespace_labels} if ctx.namespace_labels else None
    return validate_batch([ctx.policy], [ctx.new_resource], ctx.admission_info, ctx.exclude_group_role, labels,
                          device)[0][0]
