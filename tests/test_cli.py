"""The drop-in CLI surface (VAEB.py:22-38, 471-612): same args dict, flags, parsing
semantics, stdout lines and trace CSV.  The model is replaced by a host-only fake so the
epoch driver runs without a GPU."""
import numpy as np
import pytest

from vaeb_amd import cli


def test_reference_keys_and_defaults():
    ref = {'seed': (15485863, int), 'n_latent': (10, int), 'n_epochs': (2000, int), 'batch_size': (100, int),
           'L': (1, int), 'hidden_unit': (-1, int), 'learning_rate': (0.01, float), 'trace_file': ('', str),
           'save_file': ('', str), 'load_file': ('', str), 'vb_param_file': ('', str)}
    for k, v in ref.items():
        assert cli.command_line_args[k] == v
    assert cli.command_line_flags[:3] == ['continuous', 'generic_estimator', 'full_varational']


def test_parse_args_values_flags_and_unused(capsys):
    a = cli.parse_args(['--n_latent', '20', '--continuous', '--learning_rate', '0.05', '--bogus', 'x', '-L', '3'])
    assert a['n_latent'] == 20 and isinstance(a['n_latent'], int)
    assert a['learning_rate'] == 0.05
    assert a['continuous'] is True and a['generic_estimator'] is False and a['full_varational'] is False
    assert a['L'] == 1  # single-dash is not parsed (scripts/LAvsLB.sh quirk)
    out = capsys.readouterr().out
    assert "Have unused args: ['--bogus', 'x', '-L', '3']" in out


def test_print_args_format(capsys):
    cli.print_args({'a': 1})
    out = capsys.readouterr().out.splitlines()
    assert out == ['Parameters used:', '--------------------------------------', '\ta: 1',
                   '--------------------------------------']


class FakeModel:
    """Host-only stand-in with the VAEB attributes train_model uses."""
    instances = []

    def __init__(self, x_train, continuous, hidden, latent, batch_size, L, lr, generic, fv, params, **kw):
        self.N = x_train.shape[0]
        self.batch_size = batch_size
        self.orders = []
        self.kw = kw
        self.objective = kw.get("objective", "sum_prior")
        self.resumed = None
        FakeModel.instances.append(self)

    def update_epoch(self, order):
        self.orders.append(np.array(order))
        return float(-10.0 * len(order))

    def set_validation_data(self, x):
        self.nvalid = x.shape[0]

    def validate_resident(self):
        # VAEB.validate: the SGVB sum; the mean_map objective returns the mean
        return -5.0 if self.objective == "mean_map" else -5.0 * self.nvalid

    def save(self, f):
        open(f, "w").write("saved")

    def save_state(self, f):
        open(f, "w").write("state")

    def load_state(self, f):
        self.resumed = open(f).read()


def test_train_model_epoch_loop_and_trace(tmp_path, monkeypatch, capsys):
    from vaeb_amd import model
    monkeypatch.setattr(model, "VAEB", FakeModel)
    monkeypatch.chdir(tmp_path)
    trace = tmp_path / "t.csv"
    args = cli.parse_args(['--n_epochs', '2', '--trace_file', str(trace), '--synthetic', '--continuous',
                           '--save_file', str(tmp_path / 'm.mdl')])
    FakeModel.instances.clear()
    cli.train_model(args)
    m = FakeModel.instances[-1]
    assert m.N == 1500  # Frey split (VAEB.py:547-548)
    # batch order: np.random.seed(seed) then one shuffle per epoch (VAEB.py:526, 571-577)
    np.random.seed(15485863)
    o = np.arange(15)
    np.random.shuffle(o)
    assert np.array_equal(m.orders[0], o)
    np.random.shuffle(o)
    assert np.array_equal(m.orders[1], o)
    rows = trace.read_text().splitlines()
    assert rows[0] == 'num_samples,L,Lvalid'
    assert rows[1] == rows[2] == '1500,-10.0,-5.0'  # each row written twice (VAEB.py:583-593)
    assert rows[3] == rows[4] == '3000,-10.0,-5.0'
    out = capsys.readouterr().out
    assert "Epoch 0 : [Lower bound: -10.0, time:" in out
    assert "          [Lower bound on validation set: -5.0]" in out
    assert (tmp_path / 'm.mdl').read_text() == "saved"


def test_missing_dataset_raises_without_synthetic(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    with pytest.raises(FileNotFoundError):
        cli.load_dataset(False, synthetic=False)
    xt, xv = cli.load_dataset(False, synthetic=True)
    assert xt.shape == (50000, 784) and xv.shape == (10000, 784)


def test_mean_map_validation_is_not_divided_twice(tmp_path, monkeypatch, capsys):
    """--objective mean_map: validate already returns the per-row mean
    (VAEBfullbayes.py:161-165), so Lvalid is printed as is; sum_prior divides the sum by
    x_valid.shape[0] (VAEB.py:582).  Both give -5.0 here."""
    from vaeb_amd import model
    monkeypatch.setattr(model, "VAEB", FakeModel)
    monkeypatch.chdir(tmp_path)
    for obj in ("mean_map", "sum_prior"):
        args = cli.parse_args(['--n_epochs', '1', '--synthetic', '--continuous', '--objective', obj])
        cli.train_model(args)
        out = capsys.readouterr().out
        assert "          [Lower bound on validation set: -5.0]" in out, (obj, out)


def test_state_file_and_resume_file(tmp_path, monkeypatch):
    """--state_file writes the native checkpoint at the end; --resume_file loads one
    before the first epoch (keys added to the args dict, never renamed)."""
    from vaeb_amd import model
    monkeypatch.setattr(model, "VAEB", FakeModel)
    monkeypatch.chdir(tmp_path)
    (tmp_path / "r.ckpt").write_text("prev")
    args = cli.parse_args(['--n_epochs', '1', '--synthetic', '--continuous', '--state_file', str(tmp_path / "s.ckpt"),
                           '--resume_file', str(tmp_path / "r.ckpt")])
    cli.train_model(args)
    assert FakeModel.instances[-1].resumed == "prev"
    assert (tmp_path / "s.ckpt").read_text() == "state"
