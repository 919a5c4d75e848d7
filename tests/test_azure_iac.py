"""Structural checks of the Azure IaC (deploy/azure/*.bicep; no az / bicep CLI here): modules
exist, every parameter passed to a module is declared there and every required one is passed,
the parameter files only name main.bicep's parameters, and the Service Bus subscriptions and
Cosmos containers match what the services actually subscribe to and store."""
import json
import re
from pathlib import Path

AZ = Path(__file__).resolve().parent.parent / "deploy" / "azure"


def _params(text):
    """name -> has_default for every `param` of a Bicep file."""
    out = {}
    for m in re.finditer(r"^param\s+(\w+)\s+\w+(\s*=)?", text, re.M):
        out[m.group(1)] = bool(m.group(2))
    return out


def _block(text, start):
    """The {...} starting at text[start] (brace-matched)."""
    depth = 0
    for i in range(start, len(text)):
        depth += {"{": 1, "}": -1}.get(text[i], 0)
        if depth == 0:
            return text[start:i + 1]
    raise AssertionError("unbalanced braces")


def _top_keys(obj):
    keys, depth = [], 0
    for m in re.finditer(r"[{}\[\]]|(\b\w+)\s*:", obj):
        t = m.group(0)
        if t in "{[":
            depth += 1
        elif t in "}]":
            depth -= 1
        elif depth == 1 and m.group(1):
            keys.append(m.group(1))
    return keys


def test_modules_exist_and_parameters_match():
    main = (AZ / "main.bicep").read_text()
    seen = set()
    # `module x 'path' = {` or a conditional `module x 'path' = if (cond) {`
    for m in re.finditer(r"^module\s+(\w+)\s+'([^']+)'\s*=\s*(?:if\s*\([^)]*\)\s*)?\{", main, re.M):
        path = AZ / m.group(2)
        assert path.exists(), path
        seen.add(path.name)
        body = _block(main, m.end() - 1)
        pm = re.search(r"params:\s*\{", body)
        passed = set(_top_keys(_block(body, pm.end() - 1))) if pm else set()
        declared = _params(path.read_text())
        assert passed <= set(declared), (path.name, passed - set(declared))
        required = {k for k, has_default in declared.items() if not has_default}
        assert required <= passed, (path.name, required - passed)
    assert seen == {p.name for p in (AZ / "modules").glob("*.bicep")}, seen
    for f in AZ.glob("parameters.*.json"):
        names = set(json.loads(f.read_text())["parameters"])
        assert names <= set(_params(main)), (f.name, names - set(_params(main)))


def test_brackets_balance():
    for f in [AZ / "main.bicep", *(AZ / "modules").glob("*.bicep")]:
        t = re.sub(r"//.*", "", f.read_text())                   # comments, interpolations, then strings out
        t = re.sub(r"\$\{[^{}]*\}", "", t)
        t = re.sub(r"'(?:\\'|[^'])*'", "''", t)
        for a, b in ("{}", "[]", "()"):
            assert t.count(a) == t.count(b), (f.name, a)


def test_service_bus_subscriptions_match_the_services():
    from copilot_for_consensus_amd.contracts.events import ROUTING_KEYS
    from copilot_for_consensus_amd.services import processing as P
    from copilot_for_consensus_amd.services.reporting import ReportingService
    sb = (AZ / "modules" / "servicebus.bicep").read_text()
    subs = {m.group(1): set(re.findall(r"'([\w.]+)'", m.group(2)))
            for m in re.finditer(r"\{\s*name:\s*'(\w+)',\s*keys:\s*\[([^\]]*)\]\s*\}", sb)}
    want = {}
    for name, cls in (("parsing", P.ParsingService), ("chunking", P.ChunkingService),
                      ("embedding", P.EmbeddingService), ("orchestrator", P.OrchestratorService),
                      ("summarization", P.SummarizationService), ("reporting", ReportingService)):
        svc = object.__new__(cls)
        want[name] = {ROUTING_KEYS[e] for e in cls.subscriptions(svc)}
    assert subs == want
    assert "copilot.events" in sb


def test_cosmos_containers_are_the_document_collections():
    from copilot_for_consensus_amd.contracts.documents import COLLECTIONS
    cos = (AZ / "modules" / "cosmos.bicep").read_text()
    got = re.search(r"var collections = \[([^\]]*)\]", cos).group(1)
    assert set(re.findall(r"'(\w+)'", got)) == set(COLLECTIONS)


def test_deployment_scripts_write_the_secrets_the_drivers_read():
    """The JWT key pair and the Entra app credentials land under the Key Vault names the secret-
    sourced driver configs ask for (the azurekeyvault provider maps _ to -)."""
    cfg = AZ.parent / "schemas" / "configs" / "adapters" / "drivers"
    jwt = json.loads((cfg / "jwt_signer" / "local.json").read_text())["properties"]
    ms = json.loads((cfg / "oidc_providers" / "microsoft.json").read_text())["properties"]
    keys = (AZ / "modules" / "jwtkeys.bicep").read_text()
    app = (AZ / "modules" / "oidc-app.bicep").read_text()
    for field in ("private_key", "public_key"):
        if field in jwt and jwt[field].get("secret_name"):
            assert f"-n {jwt[field]['secret_name'].replace('_', '-')} " in keys, field
    for field in ("microsoft_client_id", "microsoft_client_secret"):
        assert f"-n {ms[field]['secret_name'].replace('_', '-')} " in app, field
    main = (AZ / "main.bicep").read_text()
    for mod in ("network", "privatedns", "privateendpoints", "jwtkeys", "oidc-app", "diagnostics", "dashboard"):
        assert f"'modules/{mod}.bicep'" in main, mod


def test_deployment_scripts_reach_a_private_vault():
    """With private networking the vault refuses public traffic, so both secret-writing deployment
    scripts run in the vnet's delegated subnet with a storage account that admits it; the JWT
    script fails loudly when the vault stays unreachable; the OIDC script rotates its client
    secret only near expiry and deletes the older ones (no pile-up of valid secrets)."""
    main = (AZ / "main.bicep").read_text()
    net = (AZ / "modules" / "network.bicep").read_text()
    assert "Microsoft.ContainerInstance/containerGroups" in net and "scriptsSubnetId" in net
    for mod in ("jwtkeys", "oidc-app"):
        t = (AZ / "modules" / f"{mod}.bicep").read_text()
        assert "containerSettings: empty(subnetId) ? null : { subnetIds: [ { id: subnetId } ] }" in t, mod
        assert "storageAccountSettings:" in t and "listKeys()" in t, mod
        i = main.index(f"'modules/{mod}.bicep'")
        body = _block(main, main.index("{", i))
        assert "subnetId: scriptsSubnet" in body and "storageAccountName: scriptsStorage" in body, mod
    jwt = (AZ / "modules" / "jwtkeys.bicep").read_text()
    assert 'if [ "$ok" != "1" ]' in jwt and "exit 1" in jwt
    oidc = (AZ / "modules" / "oidc-app.bicep").read_text()
    assert "RENEW_DAYS" in oidc and "az ad app credential delete" in oidc and "--expires" in oidc
    # the reset only happens in the renewal branch
    assert oidc.index("credential reset") > oidc.index("else")
